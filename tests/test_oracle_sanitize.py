"""The CPU restatement (oracle/rmr_oracle.c) under AddressSanitizer + UndefinedBehaviorSanitizer
(the build's CPU code under ASan/UBSan; GPU ASan is not available on this pool). A
sanitizer build of liboracle is preloaded into a child interpreter that renders every scene family
(RM1 node programs with refraction and volumes, RM2 NEE, RM3 spectral, Mandelbulb, the 256-primitive
union, env-map sky, separateChannels); any report fails the test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import os, sys
sys.path.insert(0, %(root)r)
from oracle import camera, oracle, scene_compile
from oracle.envmap import synthetic_env
from raymarchrenderer_amd import abi, time_schedule
G = os.path.join(%(root)r, "tests", "golden", "scenes")
S = os.path.join(%(root)r, "scenes")
cases = [(os.path.join(S, "cornell5.scene"), "rm1", {"max_bounces": 4}, False),
         (os.path.join(G, "default.scene"), "rm1", {}, False),
         (os.path.join(G, "glass_test.scene"), "rm1", {"separate_channels": 1}, False),
         (os.path.join(G, "multilight.scene"), "rm1", {}, True),
         (os.path.join(G, "simple.scene"), "rm2", {}, True),
         (None, "rm3", {}, False),
         (os.path.join(S, "mandelbulb.scene"), "rm1", {"max_bounces": 2}, False),
         (os.path.join(S, "csg256.scene"), "rm1", {"max_bounces": 2}, False)]
W, H = 12, 9
for path, var, kw, env in cases:
    t = scene_compile.compile_scene({}, var) if path is None else scene_compile.load_scene_file(path, var)
    if env:
        kw = dict(kw, use_env_tex=1)
    o = oracle.Oracle(t, abi.default_params(**kw), camera.default_view(W, H), W, H,
                      env=synthetic_env() if env else None)
    img = o.render(time_schedule(2), nthreads=1)
    assert img.shape == (H, W, 4)
print("sanitized oracle ok")
'''


def _gcc_file(name):
    return subprocess.check_output(["gcc", "-print-file-name=" + name], text=True).strip()


def test_oracle_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + r.stderr[-500:])
    env = dict(os.environ)
    env["LD_PRELOAD"] = ":".join([_gcc_file("libasan.so"), _gcc_file("libubsan.so")])
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["RMR_ORACLE_LIB"] = os.path.join(ROOT, "oracle", "_san", "liboracle_san.so")
    r = subprocess.run([sys.executable, "-c", SCRIPT % {"root": ROOT}], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert "sanitized oracle ok" in r.stdout
