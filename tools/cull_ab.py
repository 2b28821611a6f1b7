"""A/B of the JIT's exact primitive culling (RMR_JIT_CULL = 0 none, 1 boxes, 2 spheres, 3 both),
interleaved in one process; checks the images stay bitwise equal. GPU only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np  # noqa: E402
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402

G = os.path.join(ROOT, "tests", "golden", "scenes")
S = os.path.join(ROOT, "scenes")
CASES = [("cornell5", os.path.join(S, "cornell5.scene"), "rm1", 4), ("default", os.path.join(G, "default.scene"), "rm1", 16),
         ("multilight", os.path.join(G, "multilight.scene"), "rm1", 16), ("rm3", None, "rm3", 16)]
W, H, SPP, ROUNDS = 1920, 1080, 8, 3
r = Renderer(0, W, H)
r.set_jit(1)
times = time_schedule(SPP)
for name, path, var, b in CASES:
    res, img = {}, {}
    for rnd in range(ROUNDS + 1):
        for cull in (0, 1, 2, 3):
            os.environ["RMR_JIT_CULL"] = str(cull)
            if path is None:
                r.load_builtin(var)
            else:
                r.load_scene(path, var)
            r.set_params(abi.default_params(max_bounces=b))
            r.reload()
            r.reset_stats()
            r.render_spp(times)
            st = r.stats()
            if rnd:
                res.setdefault(cull, []).append(st.trace_ms)
            img[cull] = r.read_accum()
    base = img[0].view(np.uint32)
    print(json.dumps({"scene": name, **{"cull%d_ms" % c: round(float(np.median(v)), 2) for c, v in res.items()},
                      "bitwise_equal": all(np.array_equal(base, img[c].view(np.uint32)) for c in img)}), flush=True)
r.close()
