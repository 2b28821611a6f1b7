"""Graphics::Display headless (rmr_display; Graphics.cpp:356-390, createFQ 227-258, FullQuad.vs/.fs,
GL_NEAREST Graphics.h:90-91, GL_FRAMEBUFFER_SRGB + SRC_ALPHA blend Graphics.cpp:268-269).

CPU: the sRGB decision points the library uses equal the restatement's, and they reproduce the
defining formula round(255 srgb(c)) on a dense set of linear values. GPU: the kernel equals the
restatement (oracle/display.py) byte for byte over zooms, centres, partial and off-screen quads,
bounds rectangles and accumulators holding NaN, negative and > 1 values."""
import numpy as np
import pytest

from oracle import display as dref
from raymarchrenderer_amd.renderer import srgb_thresholds


def test_srgb_thresholds_library_equals_restatement():
    assert np.array_equal(srgb_thresholds().view(np.uint32), dref.srgb_thresholds().view(np.uint32))


def test_srgb_thresholds_reproduce_formula():
    rng = np.random.default_rng(3)
    c = np.concatenate([rng.uniform(0, 1, 200000), rng.uniform(0, 0.004, 20000), np.linspace(0, 1, 100001),
                        [0.0, 1.0, 0.0031308, 1e-30, 0.999, 1.5, -0.2]]).astype(np.float32)
    assert np.array_equal(dref.srgb8(c), dref.srgb8_direct(c))
    thr = dref.srgb_thresholds()
    # each decision point is the first float of its byte: the float below it is one byte lower
    below = np.nextafter(thr[1:], np.float32(0))
    assert np.array_equal(dref.srgb8(thr[1:]).astype(int) - dref.srgb8(below).astype(int), np.ones(255, int))


CASES = [
    # centre, zoom, min, max, screen (w, h)
    ((160.0, 120.0), 1.0, (0, 0), (320, 240), (320, 240)),      # 1:1, whole screen
    ((160.0, 120.0), 0.5, (1, 1), (319, 239), (320, 240)),      # the GUI's start: zoom 0.5 (GUI.cpp:187)
    ((100.3, 77.9), 2.7, (20.5, 10.0), (250.0, 200.25), (300, 220)),   # magnified, clipped by bounds
    ((-40.0, 300.0), 1.3, (0, 0), (500, 500), (256, 256)),      # quad partly off screen
    ((128.0, 96.0), 0.37, (0, 0), (1000, 1000), (257, 193)),    # minified, ragged screen
]


@pytest.mark.gpu
@pytest.mark.parametrize("centre,zoom,vmin,vmax,size", CASES)
def test_display_bytes_equal_restatement(centre, zoom, vmin, vmax, size):
    from raymarchrenderer_amd import Renderer
    W, H = 200, 150
    rng = np.random.default_rng(11)
    acc = rng.uniform(-0.2, 1.3, size=(H, W, 4)).astype(np.float32)
    acc[rng.random((H, W)) < 0.01, 0] = np.nan
    acc[..., 1] = np.where(rng.random((H, W)) < 0.3, rng.uniform(0, 0.004, (H, W)), acc[..., 1]).astype(np.float32)
    bg = rng.integers(0, 256, size=(size[1], size[0], 4), dtype=np.uint8)
    r = Renderer(0, W, H)
    try:
        r.write_accum(acc)
        got = r.display(centre, zoom, vmin, vmax, screen=bg)
    finally:
        r.close()
    want = dref.display(acc, centre, zoom, vmin, vmax, bg)
    bad = np.argwhere(got != want)
    assert bad.size == 0, "%d bytes differ, first %s: %s vs %s" % (len(bad), bad[0], got[tuple(bad[0][:2])],
                                                                  want[tuple(bad[0][:2])])


@pytest.mark.gpu
def test_display_device_buffer_matches_host_path():
    import torch
    from raymarchrenderer_amd import Renderer
    W, H = 64, 48
    acc = np.random.default_rng(2).uniform(0, 1, size=(H, W, 4)).astype(np.float32)
    r = Renderer(0, W, H)
    try:
        r.write_accum(acc)
        host = r.display((50.0, 40.0), 1.5, (0, 0), (100, 80), screen=np.zeros((80, 100, 4), np.uint8))
        dev = torch.zeros((80, 100, 4), dtype=torch.uint8, device="cuda")
        s = torch.cuda.Stream()
        r.set_stream(s.cuda_stream)
        r.display_device((50.0, 40.0), 1.5, (0, 0), (100, 80), dev, 100, 80)   # a tensor: its size
        s.synchronize()
        assert np.array_equal(dev.cpu().numpy(), host)
        dev2 = torch.zeros_like(dev)   # a raw device pointer with the buffer's size
        r.display_device((50.0, 40.0), 1.5, (0, 0), (100, 80), dev2.data_ptr(), 100, 80, nbytes=dev2.numel())
        s.synchronize()
        assert np.array_equal(dev2.cpu().numpy(), host)
        with pytest.raises(ValueError):   # a raw pointer without its size is refused (renderer.py)
            r.display_device((50.0, 40.0), 1.5, (0, 0), (100, 80), dev2.data_ptr(), 100, 80)
    finally:
        r.close()


@pytest.mark.gpu
def test_display_rejects_wrong_screen_buffers():
    """A screen that is not (h, w, 4) RGBA8 is refused before any copy (renderer.py), and the C ABI
    refuses a buffer smaller than screen_w * screen_h * 4 bytes (rmr_display / rmr_display_device)."""
    import ctypes as C
    from raymarchrenderer_amd import RMRError, Renderer
    from raymarchrenderer_amd._lib import lib
    RMR_E_INVALID = -1   # rmr.h
    r = Renderer(0, 16, 16)
    try:
        with pytest.raises(ValueError):
            r.display((8.0, 8.0), 1.0, (0, 0), (16, 16), screen=np.zeros((16, 16, 3), np.uint8))
        buf = np.zeros((16, 16, 4), np.uint8)
        rc = r.lib.rmr_display(r.ctx, 8.0, 8.0, 1.0, 0.0, 0.0, 16.0, 16.0, 16, 16, buf.ctypes.data, buf.nbytes - 1)
        assert rc == RMR_E_INVALID
        rc = r.lib.rmr_display_device(r.ctx, 8.0, 8.0, 1.0, 0.0, 0.0, 16.0, 16.0, 16, 16, C.c_void_p(1), 16 * 16 * 4 - 4)
        assert rc == RMR_E_INVALID
        with pytest.raises(RMRError):
            r.display_device((8.0, 8.0), 1.0, (0, 0), (16, 16), 1, 16, 16, nbytes=100)
    finally:
        r.close()


# ---------------------------------------------------------------------------------------------
# Pin to the reference itself: FullQuad.vs / FullQuad.fs run by Graphics::Display's GL state on
# Mesa llvmpipe (oracle/glsl_ref/display_harness.c; tests/golden/display_ref.npz, generated by
# oracle/glsl_ref/make_goldens.py --only display).
#
# What GL leaves to the implementation, and so the tolerance:
# * the float -> sRGB8 encode: llvmpipe's is approximate (0.5 -> 187 where round(255 srgb(0.5)) =
#   round(187.52) = 188): +-1 per channel;
# * which texel GL_NEAREST picks when a fragment's exact texture coordinate lies on a texel
#   boundary (zoom 0.5 or 1 with half-pixel offsets put every fragment there): the interpolated
#   coordinate's rounding decides, so there either neighbour is accepted.
# Everything else is exact: which pixels the quad covers (GL's edge rule), the FullQuad.fs bounds
# test, the blend (pixels outside keep the background byte for byte), NaN / inf / negative / > 1
# texels.
# ---------------------------------------------------------------------------------------------
def _ref_cases():
    import os
    from .conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "display_ref.npz"))
    acc = g["accum"]
    cases = []
    k = 0
    while "case%d" % k in g.files:
        c = g["case%d" % k]
        centre, zoom, vmin, vmax = (c[0], c[1]), c[2], (c[3], c[4]), (c[5], c[6])
        size = (int(c[7]), int(c[8]))
        cases.append((centre, zoom, vmin, vmax, size, g["out%d" % k]))
        k += 1
    return acc, cases


def _background(w, h):
    y, x = np.mgrid[0:h, 0:w]
    bg = np.stack([(7 * x + 13 * y) % 256, (11 * x + 3 * y + 50) % 256, (5 * x + 17 * y + 99) % 256,
                   np.full_like(x, 7)], -1)
    return bg.astype(np.uint8)


def _check_against_reference(got, ref, acc, centre, zoom, vmin, vmax, size):
    H, W = acc.shape[:2]
    bg = _background(*size)
    drawn_ref = ref[..., 3] == 255
    drawn_got = got[..., 3] == 255
    # FullQuad.fs tests the interpolated varying Pos against the bounds: a pixel centre exactly on a
    # bounds edge is decided by the interpolation's rounding (llvmpipe: either way, by case)
    px = np.arange(size[0]) + 0.5
    py = np.arange(size[1]) + 0.5
    tie = (np.isin(py, [vmin[1], vmax[1]])[:, None]) | (np.isin(px, [vmin[0], vmax[0]])[None, :])
    cov = drawn_ref != drawn_got
    assert not (cov & ~tie).any(), "coverage differs at %d pixels" % (cov & ~tie).sum()
    assert np.array_equal(got[~drawn_got], bg[~drawn_got]) and np.array_equal(ref[~drawn_ref], bg[~drawn_ref])
    drawn_ref = drawn_ref & drawn_got
    # exact texture coordinate of every pixel centre (float64), and whether it sits on a texel boundary
    hw, hh = np.float32(W / 2) * np.float32(zoom), np.float32(H / 2) * np.float32(zoom)
    x0, x1 = float(np.float32(centre[0]) - hw), float(np.float32(centre[0]) + hw)
    y0, y1 = float(np.float32(centre[1]) - hh), float(np.float32(centre[1]) + hh)
    uw = (np.arange(size[0]) + 0.5 - x0) / (x1 - x0) * W
    vh = (np.arange(size[1]) + 0.5 - y0) / (y1 - y0) * H
    on_u = np.abs(uw - np.round(uw)) < 1e-3
    on_v = np.abs(vh - np.round(vh)) < 1e-3
    thr = dref.srgb_thresholds()
    d = np.abs(got[..., :3].astype(int) - ref[..., :3].astype(int)).max(-1)
    ok = ~drawn_ref | (d <= 1)
    n_boundary = 0
    for y, x in np.argwhere(~ok):
        assert on_u[x] or on_v[y], "pixel (%d, %d): %s vs reference %s" % (x, y, got[y, x], ref[y, x])
        n_boundary += 1
        iu = [int(np.round(uw[x])) - 1, int(np.round(uw[x]))] if on_u[x] else [int(np.floor(uw[x]))]
        jv = [int(np.round(vh[y])) - 1, int(np.round(vh[y]))] if on_v[y] else [int(np.floor(vh[y]))]
        cands = [dref.srgb8(acc[j % H, i % W, :3], thr).astype(int)
                 for i in iu for j in jv]
        assert any(np.abs(c - ref[y, x, :3].astype(int)).max() <= 1 for c in cands), (x, y)
        assert any(np.abs(c - got[y, x, :3].astype(int)).max() <= 1 for c in cands), (x, y)
    return n_boundary


def test_display_restatement_vs_reference_llvmpipe():
    """oracle/display.py (the restatement rmr_display is tested against byte for byte) against the
    reference's own display pass on llvmpipe, every case."""
    acc, cases = _ref_cases()
    assert len(cases) >= 9
    exact = total = 0
    for centre, zoom, vmin, vmax, size, ref in cases:
        got = dref.display(acc, centre, zoom, vmin, vmax, _background(*size))
        _check_against_reference(got, ref, acc, centre, zoom, vmin, vmax, size)
        exact += int((got == ref).all(-1).sum())
        total += got.shape[0] * got.shape[1]
    assert exact > 0.6 * total


@pytest.mark.gpu
def test_display_kernel_vs_reference_llvmpipe():
    """rmr_display (k_display) against the reference's display pass on llvmpipe, every case."""
    from raymarchrenderer_amd import Renderer
    acc, cases = _ref_cases()
    r = Renderer(0, acc.shape[1], acc.shape[0])
    try:
        r.write_accum(acc)
        for centre, zoom, vmin, vmax, size, ref in cases:
            got = r.display(centre, zoom, vmin, vmax, screen=_background(*size))
            _check_against_reference(got, ref, acc, centre, zoom, vmin, vmax, size)
            want = dref.display(acc, centre, zoom, vmin, vmax, _background(*size))
            assert np.array_equal(got, want)
    finally:
        r.close()
