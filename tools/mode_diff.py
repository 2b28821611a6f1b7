"""Localise a bitwise difference between two settings of an environment switch read at scene load /
specialisation time (e.g. RMR_GRID 1 0): renders per-sample planes of a frame under each, lists
the differing samples, and runs the CPU oracle on the first few to say which setting is exact.

    python tools/mode_diff.py RMR_GRID 1 0 [--scene scenes/cornell5.scene] [--spp 4] [--bounces 4]
    python tools/mode_diff.py culling 7 0 --scene scenes/csg256.scene    (rmr_set_culling flags)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np  # noqa: E402
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402
from oracle import camera, oracle, scene_compile  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("var")
ap.add_argument("a")
ap.add_argument("b")
ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "cornell5.scene"), help="scene file, or 'builtin'")
ap.add_argument("--variant", default="rm1")
ap.add_argument("--spp", type=int, default=4)
ap.add_argument("--bounces", type=int, default=4)
ap.add_argument("--W", type=int, default=1920)
ap.add_argument("--H", type=int, default=1080)
ap.add_argument("--show", type=int, default=6)
a = ap.parse_args()

W, H = a.W, a.H
prm = abi.default_params(max_bounces=a.bounces)
view = camera.default_view(W, H)
times = time_schedule(a.spp)
r = Renderer(0, W, H)
r.set_jit(1)
planes = {}
for v in (a.a, a.b):
    if a.var == "culling":   # rmr_set_culling flags instead of an environment switch
        r.set_culling(int(v))
    else:
        os.environ[a.var] = v
    if a.scene == "builtin":
        r.load_builtin(a.variant)
    else:
        r.load_scene(a.scene, a.variant)
    r.set_params(prm)
    r.set_view(view)
    r.reload()
    planes[v] = r.trace_samples(times, (0, 0, W, H))
r.close()
A, B = planes[a.a], planes[a.b]
diff = np.any(A.view(np.uint32) != B.view(np.uint32), axis=-1) & ~(np.isnan(A).any(-1) & np.isnan(B).any(-1))
ks, ys, xs = np.nonzero(diff)
print("differing samples: %d of %d" % (len(ks), diff.size), flush=True)
tables = scene_compile.compile_scene({}, a.variant) if a.scene == "builtin" else scene_compile.load_scene_file(a.scene, a.variant)
orc = oracle.Oracle(tables, prm, view, W, H)
for i in range(min(a.show, len(ks))):
    k, y, x = int(ks[i]), int(ys[i]), int(xs[i])
    cpu = orc.trace_samples(times, (x, y, x + 1, y + 1))[k, 0, 0]
    print("k=%d x=%d y=%d  %s=%s  %s=%s  oracle=%s  exact: %s" % (
        k, x, y, a.a, A[k, y, x], a.b, B[k, y, x], cpu,
        [v for v, P in ((a.a, A), (a.b, B)) if np.array_equal(P[k, y, x].view(np.uint32), cpu.view(np.uint32))]), flush=True)
