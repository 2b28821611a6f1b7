"""Same-process A/B of an environment switch read when the JIT source is generated
(e.g. RMR_JIT_BAKE, RMR_JIT_CULL), or of rmr_set_culling flags (var "culling"): per scene, median
trace time per setting and a bitwise comparison of the images.

    python tools/env_ab.py culling 7 0 [--spp 16]
    python tools/env_ab.py shade_t 4 6 8         (rmr_set_tuning shading threshold)
    python tools/env_ab.py RMR_JIT_BAKE 1 0
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np  # noqa: E402
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("var")
ap.add_argument("values", nargs="+")
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--W", type=int, default=1920)
ap.add_argument("--H", type=int, default=1080)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--scenes", default="", help="comma-separated subset of the scene names")
a = ap.parse_args()

G = os.path.join(ROOT, "tests", "golden", "scenes")
CASES = [("cornell5", os.path.join(ROOT, "scenes", "cornell5.scene"), "rm1", 4),
         ("multilight", os.path.join(G, "multilight.scene"), "rm1", 16),
         ("default", os.path.join(G, "default.scene"), "rm1", 16),
         ("glass", os.path.join(G, "glass_test.scene"), "rm1", 16),
         ("rm3", None, "rm3", 16),
         ("rm2simple", os.path.join(G, "simple.scene"), "rm2", 16),
         ("csg256", os.path.join(ROOT, "scenes", "csg256.scene"), "rm1", 4),
         ("mandelbulb", os.path.join(ROOT, "scenes", "mandelbulb.scene"), "rm1", 2)]
r = Renderer(0, a.W, a.H)
r.set_jit(1)
times = time_schedule(a.spp)
for name, path, variant, b in CASES:
    if a.scenes and name not in a.scenes.split(","):
        continue
    res, tot, img = {}, {}, {}
    for rnd in range(a.rounds + 1):
        for v in a.values:
            if a.var == "culling":
                r.set_culling(int(v))
            elif a.var == "shade_t":   # shading / hand-over threshold (bits 8-15: refill threshold)
                r.set_tuning(int(v), -1, -1)
            else:
                os.environ[a.var] = v
            if path is None:
                r.load_builtin(variant)
            else:
                r.load_scene(path, variant)
            r.set_params(abi.default_params(max_bounces=b))
            r.reload()
            r.reset_stats()
            r.render_spp(times)
            st = r.stats()
            if rnd:
                res.setdefault(v, []).append(st.trace_ms)
                tot.setdefault(v, []).append(st.trace_ms + st.fold_ms)
            img[v] = r.read_accum()
    ref = img[a.values[0]].view(np.uint32)
    print(json.dumps({"scene": name, **{"%s=%s_ms" % (a.var, k): round(float(np.median(t)), 2) for k, t in res.items()},
                      **{"%s=%s_ms_with_fold" % (a.var, k): round(float(np.median(t)), 2) for k, t in tot.items()},
                      "bitwise_equal": all(np.array_equal(ref, img[v].view(np.uint32)) for v in a.values)}), flush=True)
r.close()
