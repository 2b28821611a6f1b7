"""GPU parity for paths the per-scene tests do not reach (round-2 coverage):

* C5 animated frames (BASELINE configs[4]): the live-primitive specialised kernel that a moving
  sphere switches the context to (rmr_api.cpp ensure_jit, rmr_jit.cpp) on the bench's own large-seed
  schedule time(f, s) = 1000 f + 0.016 s, bitwise against the oracle at frames 1, 37 and 90;
* sample-plane chunking (rmr_api.cpp render_tiles: launches split at the sample-plane budget) —
  several launches per frame fold to the same bits as one;
* the full C2, C3, C4, C5, RM2 and RM3 frames (1920x1080; C4 3840x2160) through the multi-GPU tile path,
  checked by properties that do not depend on size (finite, non-negative, alpha 1) and bitwise
  against the oracle on random 8x8 tiles;
* FrameRenderer's stream ordering (zero -> render -> collective on one stream) read back on that
  stream only, and rmr_render_tiles' rejection of repeated tiles.
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import camera, oracle, scene_compile
from raymarchrenderer_amd import RMRError, abi, time_schedule

from .conftest import GOLDEN, SCENES

pytestmark = pytest.mark.gpu


def _same(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def _c5_scene(frame):
    """bench.py scene_for_frame for C5: Cornell-5 with the sphere centre y = 0.5 sin(2 pi f / 120)."""
    with open(os.path.join(SCENES, "cornell5.scene")) as f:
        sc = json.load(f)
    sc["objects"][3]["nodes"][0]["inputs"][1][1] = 0.5 * math.sin(2.0 * math.pi * frame / 120.0)
    return sc


def _setup(r, scene, W, H, variant="rm1", **kw):
    r.set_image_size(W, H)
    r.reload()
    if scene is None:
        r.load_builtin(variant)
    else:
        r.load_scene(scene, variant)
    prm = abi.default_params(**kw)
    r.set_params(prm)
    view = camera.default_view(W, H)
    r.set_view(view)
    return prm, view


def test_c5_animated_frames_live_kernel_bitexact_vs_oracle(renderer):
    W, H = 64, 48
    renderer.set_jit(1)
    try:
        # frame 0 bakes the layout's kernel; every later frame moves the sphere, which makes it a
        # live (loaded) primitive of the specialised kernel while the walls stay literals
        _setup(renderer, _c5_scene(0), W, H, max_bounces=4)
        renderer.render_spp(time_schedule(1, frame=0))
        for f in (1, 37, 90):
            prm, view = _setup(renderer, _c5_scene(f), W, H, max_bounces=4)
            renderer.reset_stats()
            times = time_schedule(3, frame=f)
            renderer.render_spp(times)
            gpu = renderer.read_accum()
            assert renderer.stats().jit_launches > 0
            cpu = oracle.Oracle(scene_compile.compile_scene(_c5_scene(f), "rm1"), prm, view, W, H).render(times)
            eq = _same(gpu, cpu)
            assert eq.all(), "frame %d: %d values differ" % (f, (~eq).sum())
    finally:
        renderer.set_jit(2)


@pytest.mark.parametrize("scene,bounces", [("cornell5.scene", 4), ("csg64.scene", 3)])
def test_multichunk_sample_planes_bitexact(renderer, scene, bounces):
    """samp_budget small enough for 4 launches per render: the running mean folded launch by
    launch equals one launch of all samples, and the oracle."""
    W, H, spp = 96, 64, 10
    path = os.path.join(SCENES, scene)
    prm, view = _setup(renderer, path, W, H, max_bounces=bounces)
    times = time_schedule(spp, frame=2)
    renderer.set_jit(1)
    try:
        renderer.reset_stats()
        renderer.render_spp(times)
        one = renderer.read_accum()
        assert renderer.stats().trace_launches == 1
        plane_bytes = (W // 8) * (H // 8) * 64 * 16
        renderer.set_tuning(samp_budget=3 * plane_bytes)   # 3 samples per launch: 3 + 3 + 3 + 1
        renderer.reload()
        renderer.reset_stats()
        renderer.render_spp(times)
        many = renderer.read_accum()
        assert renderer.stats().trace_launches == 4
    finally:
        renderer.set_tuning(samp_budget=48 << 30)   # the default (rmr_api.cpp)
        renderer.set_jit(2)
    assert _same(one, many).all()
    cpu = oracle.Oracle(scene_compile.load_scene_file(path, "rm1"), prm, view, W, H).render(times)
    assert _same(many, cpu).all()


def test_full_c2_frame_properties_and_sampled_tiles(renderer):
    """The headline frame itself (C2: 1920x1080, 4 bounces; 4 spp here) through the multi-GPU tile
    path (rmr_render_tiles over the 32x32 tiles, one launch, the specialised kernel)."""
    from raymarchrenderer_amd.multi_gpu import frame_tiles
    W, H, spp = 1920, 1080, 4
    path = os.path.join(SCENES, "cornell5.scene")
    prm, view = _setup(renderer, path, W, H, max_bounces=4)
    times = time_schedule(spp)
    renderer.reset_stats()
    renderer.render_tiles(times, frame_tiles(W, H, 32), 32)
    img = renderer.read_accum()
    st = renderer.stats()
    assert st.jit_launches == st.trace_launches == 1
    assert np.isfinite(img).all()
    assert (img[..., :3] >= 0).all() and (img[..., 3] == 1.0).all()
    # the frame mean is stable at 4 spp x 2 M pixels; Cornell-5 with this camera is ~0.26
    assert 0.1 < float(img[..., :3].mean()) < 0.6
    rng = np.random.default_rng(5)
    orc = oracle.Oracle(scene_compile.load_scene_file(path, "rm1"), prm, view, W, H)
    for _ in range(6):
        x0 = int(rng.integers(0, W // 8)) * 8
        y0 = int(rng.integers(0, H // 8)) * 8
        cpu = orc.render(times, rect=(x0, y0, x0 + 8, y0 + 8))
        eq = _same(img[y0:y0 + 8, x0:x0 + 8], cpu[y0:y0 + 8, x0:x0 + 8])
        assert eq.all(), "tile (%d, %d)" % (x0, y0)


def _full_frame_check(renderer, scene, W, H, spp, bounces, frame=0, ntiles=6, seed=11,
                      mean_range=(0.0, 10.0), variant="rm1"):
    """Render a BASELINE config's full frame through rmr_render_tiles (32x32 tiles, the bench's
    path: the specialised kernel rmr_jit_trace), then check size-independent properties (finite,
    non-negative, alpha 1, a plausible frame mean) and `ntiles` random 8x8 tiles bitwise against
    the oracle (RM1:567-613 per pixel)."""
    from raymarchrenderer_amd.multi_gpu import frame_tiles
    prm, view = _setup(renderer, scene, W, H, variant=variant, max_bounces=bounces)
    times = time_schedule(spp, frame=frame)
    renderer.reset_stats()
    renderer.render_tiles(times, frame_tiles(W, H, 32), 32)
    img = renderer.read_accum()
    st = renderer.stats()
    assert st.jit_launches == st.trace_launches >= 1
    assert np.isfinite(img).all()
    assert (img[..., :3] >= 0).all() and (img[..., 3] == 1.0).all()
    m = float(img[..., :3].mean())
    assert mean_range[0] < m < mean_range[1], m
    if scene is None or isinstance(scene, dict):
        tables = scene_compile.compile_scene(scene or {}, variant)
    else:
        tables = scene_compile.load_scene_file(scene, variant)
    orc = oracle.Oracle(tables, prm, view, W, H)
    rng = np.random.default_rng(seed)
    picks = [(int(rng.integers(0, W // 8)) * 8, int(rng.integers(0, H // 8)) * 8) for _ in range(ntiles)]
    # plus two of the busiest tiles (largest radiance spread: edges, the primitives' cluster), which
    # uniform picks can miss on a mostly-empty frame
    lum = img[: H // 8 * 8, : W // 8 * 8, :3].sum(-1).reshape(H // 8, 8, W // 8, 8)
    spread = lum.std(axis=(1, 3)).ravel()
    top = np.argsort(spread)[-max(1, spread.size // 100):]
    for k in rng.choice(top, 2, replace=False):
        picks.append((int(k % (W // 8)) * 8, int(k // (W // 8)) * 8))
    for x0, y0 in picks:
        cpu = orc.render(times, rect=(x0, y0, x0 + 8, y0 + 8))
        eq = _same(img[y0:y0 + 8, x0:x0 + 8], cpu[y0:y0 + 8, x0:x0 + 8])
        assert eq.all(), "tile (%d, %d): %d values differ" % (x0, y0, (~eq).sum())
    return img, st


def test_full_c3_frame_properties_and_sampled_tiles(renderer):
    """C3 (BASELINE configs[2]): the Mandelbulb at its production size 1920x1080, 2 bounces;
    2 spp instead of 128 (the sample loop is the same code at every spp)."""
    _full_frame_check(renderer, os.path.join(SCENES, "mandelbulb.scene"), 1920, 1080, 2, 2,
                      ntiles=8, seed=31, mean_range=(0.005, 1.0))


def test_full_c4_frame_properties_and_sampled_tiles(renderer):
    """C4 (BASELINE configs[3]): the 256-primitive union at its production size 3840x2160,
    4 bounces, through the nearest-primitive cache and the candidate grid; 1 spp instead of 256.
    The tiles include ones on the sphere cluster (the grid's region)."""
    img, st = _full_frame_check(renderer, os.path.join(SCENES, "csg256.scene"), 3840, 2160, 1, 4,
                                ntiles=8, seed=41, mean_range=(0.005, 2.0))
    assert st.map_evals > 0


@pytest.mark.timeout(300)
def test_c4_production_launch_sampled_pixels_bitexact(renderer):
    """C4 exactly as the bench renders it: 3840x2160 at 256 spp, 4 bounces, all 32x32 tiles in ONE
    launch (2.12e9 units, unit indices up to 2^31 - 2^25; 34 GB of sample planes, so plane offsets far
    beyond 4 GiB; rmr_trace.h unit_pixel / fold_main). Three pixels — the frame's last one (the highest
    tile and plane offsets), the brightest and a median one — are checked bitwise against the oracle's
    running mean of all 256 samples (RM1:600-612 folds every sample in order, so each pixel is a check
    of its 256 per-sample radiances through the fold)."""
    from raymarchrenderer_amd.multi_gpu import frame_tiles
    W, H, spp = 3840, 2160, 256
    path = os.path.join(SCENES, "csg256.scene")
    prm, view = _setup(renderer, path, W, H, max_bounces=4)
    times = time_schedule(spp)
    renderer.set_jit(1)
    try:
        renderer.reset_stats()
        renderer.render_tiles(times, frame_tiles(W, H, 32), 32)
        img = renderer.read_accum()
        st = renderer.stats()
    finally:
        renderer.set_jit(2)
        renderer.set_image_size(64, 64)   # release the 34 GB of planes' frame
        renderer.reload()
    assert st.jit_launches == st.trace_launches == 1
    assert st.samples == W * H * spp
    assert np.isfinite(img).all() and (img[..., :3] >= 0).all() and (img[..., 3] == 1.0).all()
    lum = img[..., :3].sum(-1)
    flat = np.argsort(lum.ravel())
    picks = [(W - 1, H - 1), (int(flat[-1] % W), int(flat[-1] // W)), (int(flat[flat.size // 2] % W), int(flat[flat.size // 2] // W))]
    orc = oracle.Oracle(scene_compile.load_scene_file(path, "rm1"), prm, view, W, H)
    for x, y in picks:
        cpu = orc.render(times, rect=(x, y, x + 1, y + 1))
        eq = _same(img[y, x], cpu[y, x])
        assert eq.all(), "pixel (%d, %d): gpu %s oracle %s" % (x, y, img[y, x], cpu[y, x])


def test_full_c5_frame_properties_and_sampled_tiles(renderer):
    """C5 (BASELINE configs[4]): an animated frame (f = 37, the sphere moved: the live-primitive
    kernel) at 1920x1080, 4 bounces, on the bench's large-seed schedule; 2 spp instead of 512.
    Frame 0 first, so that the layout's kernel is baked and frame 37 switches it to live."""
    from raymarchrenderer_amd.multi_gpu import frame_tiles
    _setup(renderer, _c5_scene(0), 1920, 1080, max_bounces=4)
    renderer.render_tiles(time_schedule(1, frame=0), frame_tiles(1920, 1080, 32), 32)
    _full_frame_check(renderer, _c5_scene(37), 1920, 1080, 2, 4, frame=37, ntiles=6, seed=53,
                      mean_range=(0.05, 1.0))


def test_full_rm3_frame_properties_and_sampled_tiles(renderer):
    """RM3 as the reference wires it (Graphics.cpp:272; bench config rm3): the built-in scene at
    1920x1080, 16 bounces, spectral paths; 1 spp instead of 4."""
    _full_frame_check(renderer, None, 1920, 1080, 1, 16, ntiles=6, seed=61, mean_range=(0.0, 10.0),
                      variant="rm3")


def test_full_rm2_frame_properties_and_sampled_tiles(renderer):
    """RM2 (bench config rm2): simple.scene at 1920x1080, 16 bounces; 1 spp instead of 4."""
    _full_frame_check(renderer, os.path.join(GOLDEN, "scenes", "simple.scene"), 1920, 1080, 1, 16,
                      ntiles=6, seed=67, mean_range=(0.0, 10.0), variant="rm2")


def test_frame_renderer_stream_ordering_without_device_sync():
    """FrameRenderer binds each renderer to its own torch stream: zeroing, the render and the
    reduce of a frame are ordered there, so reading the frame back on that stream alone (no
    device-wide sync) sees the finished frame — twice in a row into the same buffer (the second
    frame's zeroing must not race the first frame's fold, nor the read the second fold)."""
    import torch
    from raymarchrenderer_amd import Renderer
    from raymarchrenderer_amd.multi_gpu import FrameRenderer, frame_tiles
    W, H, tile = 160, 96, 32
    path = os.path.join(SCENES, "cornell5.scene")
    tiles_all = frame_tiles(W, H, tile)
    part = np.array(tiles_all[1::2], np.int32)   # a partial tile set: the rest of the frame stays 0
    r = Renderer(0, W, H)
    ref = Renderer(0, W, H)
    try:
        for x in (r, ref):
            _setup(x, path, W, H, max_bounces=4)
        acc = torch.full((H, W, 4), 7.0, dtype=torch.float32, device="cuda")
        fr = FrameRenderer(r, acc, W, H, tile, 0, 1)
        fr.tiles = part
        for f in range(2):
            times = time_schedule(6, frame=f)
            out = fr.frame(times)
            with torch.cuda.stream(fr.streams[0]):
                got = out.to("cpu", non_blocking=False).numpy().copy()
            ref.reload()
            ref.render_tiles(times, part, tile)
            want = ref.read_accum()
            assert _same(got, want).all(), "frame %d" % f
    finally:
        r.close()
        ref.close()


def test_render_tiles_rejects_repeated_tiles(renderer):
    _setup(renderer, os.path.join(SCENES, "cornell5.scene"), 64, 64, max_bounces=1)
    with pytest.raises(RMRError):
        renderer.render_tiles(time_schedule(1), [(0, 0), (1, 0), (0, 0)], 32)
    with pytest.raises(RMRError):
        renderer.render_tiles(time_schedule(1), [(-1, 0)], 32)
    renderer.render_tiles(time_schedule(1), [(0, 0), (1, 1)], 32)


@pytest.mark.parametrize("scene", ["mandelbulb.scene", "cornell5.scene"])
def test_frame_renderer_cost_ordered_tiles_same_frame(scene):
    """FrameRenderer.order_tiles_by_cost (the bench's default tile order): the costliest tiles first by
    a probe of each tile's map() evaluations; the probe's writes into the first accumulator do not
    reach the frame, and the frame is the row-major frame bit for bit."""
    import torch
    from raymarchrenderer_amd import Renderer
    from raymarchrenderer_amd.multi_gpu import FrameRenderer, frame_tiles, tile_costs
    W, H, tile = 192, 128, 32
    path = os.path.join(SCENES, scene)
    r = Renderer(0, W, H)
    ref = Renderer(0, W, H)
    try:
        for x in (r, ref):
            _setup(x, path, W, H, max_bounces=2)
        acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        fr = FrameRenderer(r, acc, W, H, tile, 0, 1)
        rows = np.array(frame_tiles(W, H, tile), np.int32)
        reordered = fr.order_tiles_by_cost(time_schedule(2), min_spread=0.0)
        cost = tile_costs(ref, rows, tile, time_schedule(2))
        assert reordered
        assert sorted(map(tuple, fr.tiles.tolist())) == sorted(map(tuple, rows.tolist()))
        want_order = rows[np.argsort(-cost, kind="stable")]
        assert np.array_equal(fr.tiles, want_order)
        assert cost.max() > cost.min()
        times = time_schedule(4, frame=3)
        out = fr.frame(times)
        with torch.cuda.stream(fr.streams[0]):
            got = out.to("cpu", non_blocking=False).numpy().copy()
        ref.reload()
        ref.render_tiles(times, rows, tile)
        want = ref.read_accum()
        assert _same(got, want).all()
    finally:
        r.close()
        ref.close()


def test_frame_renderer_tile_order_trial_same_frame():
    """order_tiles_by_cost with trial frames (bench.py's default): two overlapping contexts render
    frames in row and cost order, the faster order is kept, and the next frame is the row-major frame
    bit for bit whichever it is."""
    import torch
    from raymarchrenderer_amd import Renderer
    from raymarchrenderer_amd.multi_gpu import FrameRenderer, frame_tiles
    W, H, tile = 192, 128, 32
    path = os.path.join(SCENES, "mandelbulb.scene")
    rs = [Renderer(0, W, H) for _ in range(2)]
    ref = Renderer(0, W, H)
    try:
        for x in rs + [ref]:
            _setup(x, path, W, H, max_bounces=2)
        accs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
        fr = FrameRenderer(rs, accs, W, H, tile, 0, 1)
        times = time_schedule(4, frame=3)
        fr.order_tiles_by_cost(time_schedule(2), min_spread=0.0, frame_times=times, trials=2)
        assert len(fr.tile_order_trial_ms) == 2 and min(fr.tile_order_trial_ms) > 0
        rows = np.array(frame_tiles(W, H, tile), np.int32)
        assert sorted(map(tuple, fr.tiles.tolist())) == sorted(map(tuple, rows.tolist()))
        out = fr.frame(times)
        fr.finish()
        torch.cuda.synchronize()
        got = out.cpu().numpy().copy()
        ref.render_tiles(times, rows, tile)
        assert _same(got, ref.read_accum()).all()
    finally:
        for x in rs + [ref]:
            x.close()
