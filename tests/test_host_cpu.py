"""Host pieces of the boundary that need no GPU: ABI surface, camera, BMP encoding, tile order."""
import ctypes as C
import math
import os
import re
import struct

import numpy as np
import pytest

from oracle import camera as ocam
from raymarchrenderer_amd import abi, camera_view, default_camera_view, encode_bmp, tile_spiral, time_schedule
from raymarchrenderer_amd._lib import EXPORTS, lib

from .conftest import ROOT


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "rmr.h")).read()
    declared = set(re.findall(r"\b(rmr_[a-z_0-9]+)\s*\(", hdr))
    L = lib()
    for name in sorted(declared):
        assert hasattr(L, name), name
    assert declared <= set(EXPORTS)


def test_abi_struct_sizes_match_ctypes():
    out = (C.c_int32 * 16)()
    n = lib().rmr_abi_sizes(out, 16)
    sizes = list(out)[:n]
    want = [C.sizeof(t) for t in (abi.Prim, abi.Op, abi.Material, abi.Spectral, abi.RM2Consts, abi.Scene,
                                  abi.Params, abi.Stats)]
    assert sizes == want
    assert sizes[0] == 48 and sizes[1] == 48


def test_default_params_are_graphics_render_uniforms():
    p = abi.Params()
    lib().rmr_default_params(C.byref(p))
    assert (p.max_dist, p.max_steps, p.max_bounces, p.step_multiply, p.separate_channels, p.use_env_tex) == \
        (1000.0, 512, 16, 0.5, 0, 0)


@pytest.mark.parametrize("W,H", [(1920, 1080), (64, 64), (1280, 720), (64, 48)])
def test_camera_matches_restatement(W, H):
    a = default_camera_view(W, H)
    b = ocam.default_view(W, H)
    np.testing.assert_allclose(a, b, rtol=0, atol=2e-7)


def test_camera_survey_values():
    # 16:9 camera-named ray00/ray01 (ray01 lands in uniform ray10)
    v = default_camera_view(1920, 1080).reshape(5, 3)
    np.testing.assert_allclose(v[1], [-0.522283256, -0.0861798972, 0.788658977], atol=2e-6)
    np.testing.assert_allclose(v[3], [-0.522283256, -0.579219222, 0.542139351], atol=2e-6)
    v1 = default_camera_view(64, 64).reshape(5, 3)
    np.testing.assert_allclose(v1[1], [-0.337071568, -0.0988779664, 0.904862642], atol=2e-6)


def _save_image_reference(rgba):
    """Graphics::SaveImage (Graphics.cpp:754-799) + SOIL/stb_image_write BMP, restated in numpy."""
    h, w = rgba.shape[:2]
    f = np.clip(rgba, 0, 1)
    u8 = np.rint(f * 255.0).astype(np.uint8)  # glReadPixels GL_UNSIGNED_BYTE (round to nearest even)
    c = u8[..., :3].astype(np.float64) / 255.0
    s = np.where(c <= 0.0031308, 12.92 * c, 1.055 * np.power(c, 1.0 / 2.4))
    s = np.clip(s, 0, 1)
    rgb = (s * 255).astype(np.uint8)
    a = u8[..., 3].astype(np.int32)
    bg = np.array([255, 0, 255], np.int32)
    px = bg + ((rgb.astype(np.int32) - bg) * a[..., None]) // 255
    px = np.where((rgb.astype(np.int32) - bg) * a[..., None] < 0,
                  bg - ((bg - rgb.astype(np.int32)) * a[..., None]) // 255, px)  # C truncates toward 0
    pad = (-w * 3) & 3
    rows = []
    for y in range(h - 1, -1, -1):
        row = px[y][:, ::-1].astype(np.uint8).tobytes() + b"\0" * pad
        rows.append(row)
    body = b"".join(rows)
    hdr = b"BM" + struct.pack("<IHHIIiiHHIIiiII", 54 + len(body), 0, 0, 54, 40, w, h, 1, 24, 0, 0, 0, 0, 0, 0)
    return hdr + body


def test_bmp_encoding_matches_saveimage(tmp_path):
    rng = np.random.default_rng(3)
    img = rng.uniform(-0.2, 1.3, size=(7, 5, 4)).astype(np.float32)
    img[..., 3] = 1.0
    img[0, 0, 3] = 0.0   # unrendered pixel: SOIL composites alpha 0 onto pink
    img[1, 1, :3] = [0.0031308 / 1.01, 0.5, 1.0]
    p = str(tmp_path / "x.bmp")
    encode_bmp(img, p)
    got = open(p, "rb").read()
    want = _save_image_reference(img)
    assert got[:54] == want[:54]
    assert got == want
    # alpha-0 pixel is pink, row 0 is the top (stored last in the bottom-up file)
    w = 5
    pad = (-w * 3) & 3
    last_row = got[54 + (7 - 1) * (w * 3 + pad):]
    assert last_row[:3] == bytes([255, 0, 255])


def test_tile_spiral_matches_program_cpp():
    # Program.cpp:113-115 start + 203-222 turns, traced by hand for the 4x4 default grid
    order = tile_spiral(4, 4)
    assert order[:6] == [(1, 1), (1, 2), (2, 2), (2, 1), (2, 0), (1, 0)]
    assert sorted(order) == sorted((x, y) for x in range(4) for y in range(4))
    # quirk kept: a non-square grid is not covered (the walk leaves the grid)
    odd = tile_spiral(3, 5)
    assert (3, 4) in odd and (0, 0) not in odd


def test_time_schedule():
    t = time_schedule(4, frame=2)
    assert t.dtype == np.float32 and t[0] == np.float32(2000.0) and t[3] == np.float32(2000.0 + 0.048)


def test_product_refuses_without_gpu_or_fails_loudly():
    # rmr_create returns an error code (not a silent CPU fallback) when no HIP device is visible
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present")
    h = C.c_void_p()
    assert lib().rmr_create(C.byref(h), 0) == -2


def test_embedded_kernel_sources_drop_comments_only():
    """csrc/tools/embed.py ships the device sources inside the library for hipRTC without their
    comments (which name diagnostic-build switches): string and character literals, preprocessor lines
    and the line numbering must survive."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "embed_mod", os.path.join(os.path.dirname(__file__), "..", "raymarchrenderer_amd", "csrc", "tools", "embed.py"))
    src = open(spec.origin).read()
    ns = {}
    exec(compile(src.split("\nout, pairs =")[0], spec.origin, "exec"), ns)   # the function, not the script
    strip = ns["strip_comments"]
    text = ('#define A 1 // a comment\nint x = 2; /* two\nlines */ int y;\n'
            'const char* s = "// not a comment /* nor this */";\nchar c = \'"\'; char d = \'\\\'\';  // tail\n'
            'printf("%d\\n", x); // RMR_JIT_OPTS\n')
    out = strip(text)
    assert out.count("\n") == text.count("\n")
    assert "comment" not in out.replace("not a comment", "")
    assert "RMR_JIT_OPTS" not in out and "tail" not in out
    assert '"// not a comment /* nor this */"' in out
    assert "char c = '\"';" in out and "char d = '\\'';" in out
    assert "#define A 1" in out and "int y;" in out and 'printf("%d\\n", x);' in out
    # a block comment is one space (`int/**/x` stays two tokens), and a multi-line one inside a macro
    # keeps the macro going (escaped line breaks)
    assert strip("int/**/x;") == "int x;"
    mac = "#define M(a) (a) /* two\nlines */ + 1\nint z = M(2);\n"
    got = strip(mac)
    assert got.count("\n") == mac.count("\n")
    assert got.splitlines()[0].endswith("\\") and "+ 1" in got.splitlines()[1]
    assert strip("int a; /* x\ny */ int b;\n") == "int a;\n int b;\n"


def test_group_library_exports_every_header_symbol():
    """librmr_group.so (include/rmr_group.h): the multi-GPU device group of the C++ host."""
    from raymarchrenderer_amd.group import GROUP_EXPORTS, group_lib
    hdr = open(os.path.join(ROOT, "include", "rmr_group.h")).read()
    declared = set(re.findall(r"\b(rmr_group_[a-z_0-9]+)\s*\(", hdr))
    L = group_lib()
    for name in sorted(declared):
        assert hasattr(L, name), name
    assert declared == set(GROUP_EXPORTS)


@pytest.mark.parametrize("W,H,tile,n", [(1920, 1080, 32, 8), (1920, 1080, 32, 3), (3840, 2160, 64, 8),
                                         (64, 48, 16, 2), (100, 70, 32, 5), (8, 8, 32, 4)])
def test_group_partition_equals_tile_partition(W, H, tile, n):
    """The C++ group's partition (rmr_group_partition) is multi_gpu.tile_partition, member by member:
    the single-process group and the one-process-per-GPU path split a frame the same way."""
    from raymarchrenderer_amd.group import group_partition
    from raymarchrenderer_amd.multi_gpu import frame_tiles, tile_partition
    seen = []
    for m in range(n):
        got = group_partition(W, H, tile, m, n)
        want = tile_partition(W, H, tile, m, n)
        assert got.shape == want.shape and (got == want).all()
        seen += [tuple(t) for t in got]
    assert sorted(seen) == sorted(frame_tiles(W, H, tile))   # every tile once


def test_group_partition_rejects_bad_arguments():
    from raymarchrenderer_amd.group import group_lib
    L = group_lib()
    for args in [(0, 10, 32, 0, 1), (10, 10, 0, 0, 1), (10, 10, 32, 1, 1), (10, 10, 32, -1, 2), (10, 10, 32, 0, 0)]:
        assert L.rmr_group_partition(*args, None, 0) < 0
