"""The multi-GPU device group of the C++ host (librmr_group.so, include/rmr_group.h) on the box's GPU.

A one-device group runs the whole group path — the tile partition, two contexts on two streams per
device, the per-frame zeroing and the RCCL reduce (ncclCommInitAll with one rank; the reduce is then an
in-place identity) — and must give the bits of a one-context render of the same frame. rmr_cli --gpus 1
(Graphics::setDevices / RenderFrame) must write the BMP the tile loop writes."""
import os
import subprocess

import numpy as np
import pytest

from raymarchrenderer_amd import Renderer, abi, time_schedule
from raymarchrenderer_amd.group import DeviceGroup

from .conftest import ROOT, SCENES
from .test_gpu_parity import same_bits

pytestmark = pytest.mark.gpu

CORNELL = os.path.join(SCENES, "cornell5.scene")
CLI = os.path.join(ROOT, "raymarchrenderer_amd", "rmr_cli")


@pytest.mark.parametrize("tile", [32, 16])
def test_group_frames_bitwise_one_context(tile):
    W, H = 72, 40   # ragged against both tile sizes
    prm = abi.default_params(max_bounces=4)
    g = DeviceGroup([0], W, H, tile=tile)
    r = Renderer(0, W, H)
    try:
        g.load_scene(CORNELL, "rm1")
        g.set_params(prm)
        g.reload()
        r.load_scene(CORNELL, "rm1")
        r.set_params(prm)
        frames = [time_schedule(3, frame=f) for f in range(3)]   # frames alternate the two contexts
        for f, times in enumerate(frames):
            g.render_frame(times)
            got = g.read_frame()
            r.reload()
            r.render_spp(times)
            want = r.read_accum()
            assert same_bits(got, want).all(), "frame %d" % f
        # pipelined: several frames in flight, the last one read
        for times in frames:
            g.render_frame(times)
        assert same_bits(g.read_frame(), want).all()
        st = g.stats(0)
        assert st.trace_launches >= 6 and st.map_evals > 0
    finally:
        g.close()
        r.close()


def test_group_rejects_repeated_devices_and_render_before_reload():
    with pytest.raises(Exception):
        DeviceGroup([0, 0], 16, 16)
    g = DeviceGroup([0], 16, 16)
    try:
        g.load_scene(CORNELL, "rm1")
        with pytest.raises(Exception) as e:
            g.render_frame(time_schedule(1))
        assert "reload" in str(e.value)
    finally:
        g.close()


@pytest.mark.parametrize("extra", [["--gpus", "1"], ["--devices", "0"]])
def test_cli_device_group_matches_tile_loop(tmp_path, extra):
    """rmr_cli through the device group (one process, RCCL) writes the tile loop's image."""
    if not os.path.exists(CLI):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "raymarchrenderer_amd", "host")])
    base = [CLI, "--scene", CORNELL, "--size", "64x48", "--samples", "3", "--bounces", "3", "--quiet"]
    a, b = tmp_path / "loop.bmp", tmp_path / "group.bmp"
    p1 = subprocess.run(base + ["--out", str(a)], capture_output=True, text=True, timeout=300)
    p2 = subprocess.run(base + ["--out", str(b)] + extra, capture_output=True, text=True, timeout=300)
    assert p1.returncode == 0, p1.stderr
    assert p2.returncode == 0, p2.stderr
    assert a.read_bytes() == b.read_bytes()
