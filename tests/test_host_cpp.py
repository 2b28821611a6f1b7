"""C++ host facades (raymarchrenderer_amd/host: Graphics / Camera / Screen over the C ABI) and the
headless driver rmr_cli (Program.cpp main loop + CLI.cpp commands of the reference)."""
import os
import subprocess

import numpy as np
import pytest

from raymarchrenderer_amd import camera_view, tile_spiral, time_schedule

from .conftest import ROOT, SCENES, has_gpu

CLI = os.path.join(ROOT, "raymarchrenderer_amd", "rmr_cli")


@pytest.fixture(scope="module")
def cli():
    if not os.path.exists(CLI):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "raymarchrenderer_amd", "host")])
    return CLI


def run(cli, *args, stdin=None, cwd=None, timeout=300):
    return subprocess.run([cli, *args], input=stdin, capture_output=True, text=True, cwd=cwd, timeout=timeout)


@pytest.mark.parametrize("grid", [(4, 4), (4, 3), (1, 1), (5, 5), (2, 2), (3, 2), (6, 6)])
def test_cli_spiral_order_matches_program_cpp(cli, grid):
    p = run(cli, "--print-tiles", "--grid", "%dx%d" % grid)
    assert p.returncode == 0
    got = [tuple(int(v) for v in ln.split()) for ln in p.stdout.strip().splitlines()]
    assert got == [tuple(t) for t in tile_spiral(*grid)]


@pytest.mark.parametrize("size", [(1920, 1080), (64, 48), (256, 256)])
def test_cli_camera_rays_follow_setview_swap(cli, size):
    """Camera::calculateRays names (ray00, ray10, ray01, ray11); Graphics::setView(eye, ray00, ray10,
    ray01, ray11) (Camera.cpp:101) puts the camera's ray10 into uniform ray01."""
    p = run(cli, "--print-view", "--size", "%dx%d" % size)
    assert p.returncode == 0
    r = np.array([[float(v) for v in ln.split()] for ln in p.stdout.strip().splitlines()], np.float32)
    m = np.sqrt(45.0)
    u = camera_view((0, 4, -6), (0, -3 / m, 6 / m), size[0] / size[1],
                    float(np.float32(3.141592653) / np.float32(4))).reshape(5, 3)
    np.testing.assert_array_equal(r[0], u[1])   # ray00
    np.testing.assert_array_equal(r[1], u[2])   # camera ray10 -> uniform ray01
    np.testing.assert_array_equal(r[2], u[3])   # camera ray01 -> uniform ray10
    np.testing.assert_array_equal(r[3], u[4])   # ray11


def test_cli_rejects_bad_arguments(cli):
    assert run(cli, "--size", "axb").returncode == 2
    assert run(cli, "--variant", "rm9").returncode == 2
    assert run(cli, "--bogus").returncode == 2


@pytest.mark.skipif(has_gpu(), reason="checks the no-device failure")
def test_cli_fails_loudly_without_gpu(cli, tmp_path):
    p = run(cli, "--scene", os.path.join(SCENES, "cornell5.scene"), "--size", "16x16", "--samples", "1",
            "--out", str(tmp_path / "x.bmp"))
    assert p.returncode == 3
    assert "no HIP device" in p.stderr
    assert not (tmp_path / "x.bmp").exists()


# ---------------------------------------------------------------------------------------------
# GPU: the C++ driver renders bitwise what the Python Renderer renders on the same schedule
# ---------------------------------------------------------------------------------------------
def _python_bmp(path, W, H, nspp, bounces=4):
    from raymarchrenderer_amd import Renderer, abi, default_camera_view
    r = Renderer(0, W, H)
    try:
        r.load_scene(os.path.join(SCENES, "cornell5.scene"), "rm1")
        r.set_params(abi.default_params(max_bounces=bounces))
        r.set_view(default_camera_view(W, H))
        r.render_spp(time_schedule(nspp))
        r.save_bmp(str(path))
    finally:
        r.close()
    return open(path, "rb").read()


@pytest.mark.gpu
def test_cli_fixed_spp_matches_python_renderer(cli, tmp_path):
    W, H, n = 64, 48, 3
    ref = _python_bmp(tmp_path / "py.bmp", W, H, n)
    base = ["--scene", os.path.join(SCENES, "cornell5.scene"), "--size", "%dx%d" % (W, H), "--samples", str(n),
            "--grid", "2x2", "--bounces", "4", "--quiet"]
    a = run(cli, *base, "--out", str(tmp_path / "a.bmp"))
    assert a.returncode == 0, a.stderr
    b = run(cli, *base, "--per-sample", "--out", str(tmp_path / "b.bmp"))
    assert b.returncode == 0, b.stderr
    assert open(tmp_path / "a.bmp", "rb").read() == ref
    assert open(tmp_path / "b.bmp", "rb").read() == ref


@pytest.mark.gpu
def test_cli_progressive_checkpoint_resume(cli, tmp_path):
    W, H = 64, 48
    ref = _python_bmp(tmp_path / "py.bmp", W, H, 3)
    base = ["--scene", os.path.join(SCENES, "cornell5.scene"), "--size", "%dx%d" % (W, H), "--samples", "0",
            "--grid", "4x4", "--bounces", "4", "--quiet"]  # square: the reference spiral skips tiles of non-square grids
    a = run(cli, *base, "--passes", "2", "--checkpoint", str(tmp_path / "ck.acc"), "--out", str(tmp_path / "a.bmp"))
    assert a.returncode == 0, a.stderr
    b = run(cli, *base, "--passes", "1", "--resume", str(tmp_path / "ck.acc"), "--out", str(tmp_path / "b.bmp"))
    assert b.returncode == 0, b.stderr
    assert open(tmp_path / "b.bmp", "rb").read() == ref


@pytest.mark.gpu
def test_cli_interactive_commands(cli, tmp_path):
    W, H = 64, 48
    ref = _python_bmp(tmp_path / "py.bmp", W, H, 2)
    names = sorted(n for n in os.listdir(SCENES) if n.endswith(".scene"))
    idx = names.index("cornell5.scene")
    cmds = "samples\n2\ngrid_width\n2\ngrid_height\n2\nload_scene\n%d\nrender\nsave\nquit\n" % idx
    p = run(cli, "--interactive", "--scene-dir", SCENES, "--size", "%dx%d" % (W, H), "--bounces", "4", "--quiet",
            "--out", str(tmp_path / "i.bmp"), stdin=cmds)
    assert p.returncode == 0, p.stderr
    assert "Saved image as" in p.stdout
    assert open(tmp_path / "i.bmp", "rb").read() == ref
