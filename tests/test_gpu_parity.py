"""GPU parity: librmr.so (HIP, gfx950) against the CPU oracle, through the C ABI.

The kernels and oracle/ implement the same float semantics (oracle/detmath.h, csrc/rmr_math.h),
so every per-sample radiance and every running-mean accumulator value must be bitwise identical
(NaN compared as NaN). Scenes: the reference's own scene files (tests/golden/scenes) and the
SURVEY §8d configs (scenes/).
"""
import os

import numpy as np
import pytest

from oracle import camera, oracle, scene_compile
from oracle.envmap import synthetic_env
from raymarchrenderer_amd import abi, time_schedule

from .conftest import GOLDEN, SCENES

pytestmark = pytest.mark.gpu

CASES = [
    # name, scene path (None = built-in), variant, params overrides
    ("rm3_builtin", None, "rm3", {}),
    ("rm3_b2", None, "rm3", {"max_bounces": 2}),
    ("rm2_simple", os.path.join(GOLDEN, "scenes", "simple.scene"), "rm2", {}),
    ("rm2_simple_b1", os.path.join(GOLDEN, "scenes", "simple.scene"), "rm2", {"max_bounces": 1}),
    ("rm1_default", os.path.join(GOLDEN, "scenes", "default.scene"), "rm1", {}),
    ("rm1_glass", os.path.join(GOLDEN, "scenes", "glass_test.scene"), "rm1", {}),
    ("rm1_multilight", os.path.join(GOLDEN, "scenes", "multilight.scene"), "rm1", {}),
    ("rm1_cornell5_b4", os.path.join(SCENES, "cornell5.scene"), "rm1", {"max_bounces": 4}),
    ("rm1_sphere1_b1", os.path.join(SCENES, "sphere1.scene"), "rm1", {"max_bounces": 1}),
    ("rm1_default_sepch", os.path.join(GOLDEN, "scenes", "default.scene"), "rm1", {"separate_channels": 1}),
    ("rm1_cornell5_steps", os.path.join(SCENES, "cornell5.scene"), "rm1", {"max_bounces": 3, "max_steps": 40}),
    ("rm1_mandelbulb_b2", os.path.join(SCENES, "mandelbulb.scene"), "rm1", {"max_bounces": 2}),
    ("rm1_csg256_b4", os.path.join(SCENES, "csg256.scene"), "rm1", {"max_bounces": 4}),
    ("rm1_sphere1_env", os.path.join(SCENES, "sphere1.scene"), "rm1", {"max_bounces": 4, "use_env_tex": 1}),
    ("rm1_default_env", os.path.join(GOLDEN, "scenes", "default.scene"), "rm1", {"use_env_tex": 1}),
    ("rm2_simple_env", os.path.join(GOLDEN, "scenes", "simple.scene"), "rm2", {"use_env_tex": 1}),
    # edge cases: zero bounces (trace() returns its throughput untouched), zero march steps (every
    # march falls out of its loop: a miss), an empty scene, separateChannels on RM2
    ("rm1_cornell5_b0", os.path.join(SCENES, "cornell5.scene"), "rm1", {"max_bounces": 0}),
    ("rm1_cornell5_steps0", os.path.join(SCENES, "cornell5.scene"), "rm1", {"max_steps": 0}),
    ("rm1_empty", os.path.join(SCENES, "empty.scene"), "rm1", {}),
    ("rm2_simple_sepch", os.path.join(GOLDEN, "scenes", "simple.scene"), "rm2", {"separate_channels": 1}),
    # separateChannels on the HO fast kernel (escape bound + approximate map per channel trace)
    ("rm1_cornell5_sepch", os.path.join(SCENES, "cornell5.scene"), "rm1", {"separate_channels": 1, "max_bounces": 4}),
    # RM1's object node set (op_union / op_subtract / op_intersect / domain_repeat / math / misc,
    # RayMarch.glsl:121-215) through the node interpreter; the 64-primitive cut of C4's generator
    # through the BVH + nearest-primitive cache
    ("rm1_csg_nodes_b4", os.path.join(SCENES, "csg_nodes.scene"), "rm1", {"max_bounces": 4}),
    ("rm1_csg64_b4", os.path.join(SCENES, "csg64.scene"), "rm1", {"max_bounces": 4}),
]


def _tables(path, variant):
    if path is None:
        return scene_compile.compile_scene({}, variant)
    return scene_compile.load_scene_file(path, variant)


def _setup(r, path, variant, W, H, overrides):
    r.set_image_size(W, H)
    r.reload()
    if path is None:
        r.load_builtin(variant)
    else:
        r.load_scene(path, variant)
    prm = abi.default_params(**overrides)
    r.set_params(prm)
    view = camera.default_view(W, H)
    r.set_view(view)
    r.set_env_map(synthetic_env() if prm.use_env_tex else None)
    return prm, view


def same_bits(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    both_nan = np.isnan(a) & np.isnan(b)
    return (a.view(np.uint32) == b.view(np.uint32)) | both_nan


@pytest.mark.parametrize("name,path,variant,overrides", CASES, ids=[c[0] for c in CASES])
def test_samples_bitexact(renderer, name, path, variant, overrides):
    W, H = 44, 36                      # ragged: not a multiple of the 8x8 tile
    rect = (3, 2, 41, 35)
    prm, view = _setup(renderer, path, variant, W, H, overrides)
    times = time_schedule(3, frame=1)
    gpu = renderer.trace_samples(times, rect)
    orc = oracle.Oracle(_tables(path, variant), prm, view, W, H, env=synthetic_env() if prm.use_env_tex else None)
    cpu = orc.trace_samples(times, rect)
    eq = same_bits(gpu[..., :3], cpu[..., :3])
    bad = np.argwhere(~eq.all(axis=-1))
    assert bad.size == 0, "%s: %d/%d samples differ; first %s gpu=%s cpu=%s" % (
        name, len(bad), eq.shape[0] * eq.shape[1] * eq.shape[2], bad[0], gpu[tuple(bad[0])], cpu[tuple(bad[0])])


@pytest.mark.parametrize("kernel", [0, 1], ids=["persistent", "per_path"])
def test_running_mean_bitexact(renderer, kernel):
    """rmr_render_spp == nspp Graphics::Render running-mean updates (RM1:600-612), both kernels."""
    W, H = 40, 24
    path = os.path.join(SCENES, "cornell5.scene")
    prm, view = _setup(renderer, path, "rm1", W, H, {"max_bounces": 4})
    renderer.set_kernel(kernel)
    try:
        times = time_schedule(5)
        renderer.render_spp(times[:2], rect=(0, 0, W, H), first_sample=0)
        renderer.render_spp(times[2:], rect=(0, 0, W, H), first_sample=2)
        gpu = renderer.read_accum()
    finally:
        renderer.set_kernel(0)
    orc = oracle.Oracle(_tables(path, "rm1"), prm, view, W, H)
    cpu = orc.render(times)
    assert same_bits(gpu, cpu).all()


def test_render_single_sample_bounds(renderer):
    """Graphics::Render(time, min, max, n) touches exactly the pixels with min <= pix < max."""
    W, H = 32, 32
    path = os.path.join(SCENES, "cornell5.scene")
    prm, view = _setup(renderer, path, "rm1", W, H, {"max_bounces": 2})
    renderer.render(0.5, (4.5, 3.0), (20.0, 17.2), 0)
    renderer.render(0.75, (4.5, 3.0), (20.0, 17.2), 1)
    gpu = renderer.read_accum()
    orc = oracle.Oracle(_tables(path, "rm1"), prm, view, W, H)
    cpu = orc.render(np.array([0.5, 0.75], np.float32), rect=(5, 3, 20, 18))
    assert same_bits(gpu, cpu).all()
    assert (gpu[:3, :, :] == 0).all() and (gpu[:, :5, :] == 0).all()
    assert (gpu[3:18, 5:20, 3] == 1).all()


@pytest.mark.parametrize("W,H", [(1, 1), (7, 3), (9, 17)])
def test_tiny_and_ragged_images(renderer, W, H):
    """Images smaller than one 8x8 tile or not a multiple of it: only in-image pixels are written."""
    path = os.path.join(SCENES, "cornell5.scene")
    prm, view = _setup(renderer, path, "rm1", W, H, {"max_bounces": 2})
    times = time_schedule(3)
    renderer.render_spp(times)
    gpu = renderer.read_accum()
    cpu = oracle.Oracle(_tables(path, "rm1"), prm, view, W, H).render(times)
    assert gpu.shape == (H, W, 4)
    assert same_bits(gpu, cpu).all()


def test_rect_clipping_and_empty_calls(renderer):
    """A rect reaching outside the image is clipped; zero samples or an empty rect is a no-op."""
    W, H = 24, 16
    path = os.path.join(SCENES, "cornell5.scene")
    prm, view = _setup(renderer, path, "rm1", W, H, {"max_bounces": 2})
    times = time_schedule(2)
    renderer.render_spp(times[:0])
    renderer.render_spp(times, rect=(5, 5, 5, 9))
    assert (renderer.read_accum() == 0).all()
    renderer.render_spp(times, rect=(-8, 10, 40, 30))
    gpu = renderer.read_accum()
    cpu = oracle.Oracle(_tables(path, "rm1"), prm, view, W, H).render(times, rect=(0, 10, W, H))
    assert same_bits(gpu, cpu).all()


def test_render_tiles_partition_sums_to_full(renderer):
    """Tile-partitioned renders (the multi-GPU unit) add up exactly to the full frame."""
    W, H = 48, 40
    path = os.path.join(SCENES, "cornell5.scene")
    _setup(renderer, path, "rm1", W, H, {"max_bounces": 2})
    times = time_schedule(2)
    renderer.render_spp(times)
    full = renderer.read_accum()
    tiles = [(tx, ty) for ty in range((H + 15) // 16) for tx in range((W + 15) // 16)]
    parts = []
    for part in (tiles[0::2], tiles[1::2]):
        renderer.reload()
        renderer.render_tiles(times, part, 16)
        parts.append(renderer.read_accum())
    assert same_bits(parts[0] + parts[1], full).all()


def test_stats_count_map_evals(renderer):
    W, H = 32, 32
    path = os.path.join(SCENES, "cornell5.scene")
    prm, view = _setup(renderer, path, "rm1", W, H, {"max_bounces": 4})
    renderer.reset_stats()
    times = time_schedule(2)
    renderer.render_spp(times)
    st = renderer.stats()
    orc = oracle.Oracle(_tables(path, "rm1"), prm, view, W, H)
    orc.render(times)
    # the kernels evaluate getNormal once per hit (the reference calls it per material node), as the
    # oracle does; on sphere/box scenes a march past the escape bound (rmr_trace.h ray_exit) ends
    # as its miss without the remaining map() calls, so the kernels count fewer
    assert 0.5 * orc.map_evals < st.map_evals <= orc.map_evals
    assert st.flops_per_map == 106
    assert st.trace_ms > 0


@pytest.mark.gpu
def test_stats_count_map_evals_exact_without_escape_bound(renderer):
    """With the work-skipping paths off every march runs every step: the count equals the oracle's
    (a node-program-material scene, glass). With them on (the escape bound covers these kernels
    since round 3) the count is lower and the image the same bit for bit."""
    W, H = 24, 24
    path = os.path.join(GOLDEN, "scenes", "glass_test.scene")
    prm, view = _setup(renderer, path, "rm1", W, H, {"max_bounces": 4})
    times = time_schedule(2)
    evals, img = {}, {}
    try:
        for flags in (0, abi.CULL_ALL):
            renderer.set_culling(flags)
            renderer.reload()
            renderer.reset_stats()
            renderer.render_spp(times)
            evals[flags] = renderer.stats().map_evals
            img[flags] = renderer.read_accum()
    finally:
        renderer.set_culling(abi.CULL_ALL)
    orc = oracle.Oracle(_tables(path, "rm1"), prm, view, W, H)
    orc.render(times)
    assert evals[0] == orc.map_evals
    assert evals[abi.CULL_ALL] < evals[0]
    assert np.array_equal(img[0].view(np.uint32), img[abi.CULL_ALL].view(np.uint32))


@pytest.mark.parametrize("scene", ["cornell5.scene", "csg256.scene"])
def test_far_camera_bitexact(renderer, scene):
    """A camera 400 units away: larger escape-box inflation (|eye| term), long primary marches
    through empty space, the nearest-primitive cache far from the scene."""
    import math
    W, H = 40, 30
    path = os.path.join(SCENES, scene)
    prm, _ = _setup(renderer, path, "rm1", W, H, {"max_bounces": 3})
    eye = (30.0, 60.0, -400.0)
    d = (-30.0, -59.0, 400.0)
    m = math.sqrt(sum(x * x for x in d))
    view = camera.view_uniforms(eye, tuple(x / m for x in d), W / H, camera.F(3.141592653) / camera.F(24))
    renderer.set_view(view)
    rect = (0, 0, W, H)
    times = time_schedule(3, frame=4)
    renderer.set_jit(1)
    try:
        gpu = renderer.trace_samples(times, rect)
    finally:
        renderer.set_jit(2)
    cpu = oracle.Oracle(_tables(path, "rm1"), prm, view, W, H).trace_samples(times, rect)
    eq = same_bits(gpu[..., :3], cpu[..., :3])
    assert eq.all(), "%d samples differ" % (~eq.all(axis=-1)).sum()


@pytest.mark.gpu
@pytest.mark.parametrize("sepch", [0, 1])
def test_eye_first_step_switch_bitexact(renderer, sepch):
    """RMR_CULL_EYE (rmr_trace.h eye_map): every primary ray's first march step from one map(eye)
    per wave. Same image bit for bit with the switch on and off (separateChannels restarts too), and
    at most one map() call fewer per primary ray (rays that escape at once never march)."""
    W, H, spp = 64, 48, 4
    path = os.path.join(SCENES, "cornell5.scene")
    _setup(renderer, path, "rm1", W, H, {"max_bounces": 4, "separate_channels": sepch})
    times = time_schedule(spp)
    img, evals = {}, {}
    try:
        for flags in (abi.CULL_ALL, abi.CULL_ALL & ~abi.CULL_EYE):
            renderer.set_culling(flags)
            renderer.reload()
            renderer.reset_stats()
            renderer.render_spp(times)
            img[flags] = renderer.read_accum()
            evals[flags] = renderer.stats().map_evals
    finally:
        renderer.set_culling(abi.CULL_ALL)
    on, off = abi.CULL_ALL, abi.CULL_ALL & ~abi.CULL_EYE
    assert np.array_equal(img[on].view(np.uint32), img[off].view(np.uint32))
    rays = W * H * spp * (3 if sepch else 1)
    assert 0 < evals[off] - evals[on] <= rays
