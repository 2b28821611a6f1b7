"""Node-program-material kernels (RM1 with mat_func node programs: default / glass_test / multilight)
built at forced occupancy targets (-DRMR_PROG_WAVES=N through the diagnostic library's RMR_JIT_OPTS).

Round 4 found the glass_test kernel at 6 / 7 waves per SIMD wrong in ~6% of its samples (the units a
wave hands out without fetching a chunk started with the previous path's throughput). The cause was
undefined behaviour in the kernel, not the compiler: `Lane L;` left most fields uninitialised, so the
optimised IR carried `phi [undef, %entry]` for every lane field at the loop header, and the register
allocator's VGPR live-range splitting (SIOptimizeVGPRLiveRange) was entitled to treat those values as
dead on the paths that came from the entry. With the lane value-initialised (rmr_trace.h trace_main)
the IR has no undef PHI left, and these builds must be bitwise equal to the oracle.

The sizes are the ones that exposed the fault: 256 x 96 at 4 spp and 16 bounces (two 128-unit work
chunks per wave of the grid, so both the fetch and the no-fetch refill paths run many times)."""
import os

import numpy as np
import pytest

from oracle import camera, oracle, scene_compile
from raymarchrenderer_amd import Renderer, abi, time_schedule

from .conftest import GOLDEN

SCENES = ["glass_test", "default", "multilight"]


@pytest.fixture(scope="module")
def diag_renderer():
    r = Renderer(0, 256, 96, diag=True)
    yield r
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [6, 7])
@pytest.mark.parametrize("scene", SCENES)
def test_prog_kernel_forced_waves_bitexact_vs_oracle(diag_renderer, monkeypatch, scene, waves):
    W, H, spp, bounces = 256, 96, 4, 16
    path = os.path.join(GOLDEN, "scenes", scene + ".scene")
    monkeypatch.setenv("RMR_JIT_OPTS", "-DRMR_PROG_WAVES=%d" % waves)
    r = diag_renderer
    r.set_jit(1)
    r.load_scene(path, "rm1")
    prm = abi.default_params(max_bounces=bounces)
    r.set_params(prm)
    view = camera.default_view(W, H)
    r.set_view(view)
    r.reload()
    r.reset_stats()
    times = time_schedule(spp)
    gpu = r.trace_samples(times, (0, 0, W, H))
    assert r.stats().jit_launches > 0
    cpu = oracle.Oracle(scene_compile.load_scene_file(path, "rm1"), prm, view, W, H).trace_samples(times, (0, 0, W, H))
    a, b = gpu[..., :3], cpu[..., :3]
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    bad = int((~same.all(-1)).sum())
    assert bad == 0, "%s at %d waves: %d of %d samples differ from the oracle" % (scene, waves, bad, same.shape[0] * same.shape[1] * same.shape[2])
