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
        r.display_device((50.0, 40.0), 1.5, (0, 0), (100, 80), dev.data_ptr(), 100, 80)
        s.synchronize()
        assert np.array_equal(dev.cpu().numpy(), host)
    finally:
        r.close()


@pytest.mark.gpu
def test_display_rejects_wrong_screen_buffers():
    """A screen that is not (h, w, 4) RGBA8 is refused before any copy (renderer.py), and the C ABI
    refuses a buffer smaller than screen_w * screen_h * 4 bytes (rmr_display / rmr_display_device)."""
    import ctypes as C
    from raymarchrenderer_amd import RMRError, Renderer, abi
    from raymarchrenderer_amd._lib import lib
    r = Renderer(0, 16, 16)
    try:
        with pytest.raises(ValueError):
            r.display((8.0, 8.0), 1.0, (0, 0), (16, 16), screen=np.zeros((16, 16, 3), np.uint8))
        buf = np.zeros((16, 16, 4), np.uint8)
        rc = lib().rmr_display(r.ctx, 8.0, 8.0, 1.0, 0.0, 0.0, 16.0, 16.0, 16, 16, buf.ctypes.data, buf.nbytes - 1)
        assert rc == abi.RMR_E_INVALID
        rc = lib().rmr_display_device(r.ctx, 8.0, 8.0, 1.0, 0.0, 0.0, 16.0, 16.0, 16, 16, C.c_void_p(1), 16 * 16 * 4 - 4)
        assert rc == abi.RMR_E_INVALID
        with pytest.raises(RMRError):
            r.display_device((8.0, 8.0), 1.0, (0, 0), (16, 16), 1, 16, 16, nbytes=100)
    finally:
        r.close()
