"""A/B of the JIT's baked literals vs structure-only primitive loads (RMR_JIT_BAKE), one process."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np  # noqa: E402
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402

r = Renderer(0, 1920, 1080)
r.set_jit(1)
times = time_schedule(16)
for name, path, b in [("cornell5", os.path.join(ROOT, "scenes", "cornell5.scene"), 4),
                      ("multilight", os.path.join(ROOT, "tests", "golden", "scenes", "multilight.scene"), 16)]:
    res, img = {}, {}
    for rnd in range(5):
        for bake in (1, 0):
            os.environ["RMR_JIT_BAKE"] = str(bake)
            r.load_scene(path, "rm1")
            r.set_params(abi.default_params(max_bounces=b))
            r.reload()
            r.reset_stats()
            r.render_spp(times)
            st = r.stats()
            if rnd:
                res.setdefault(bake, []).append(st.trace_ms)
            img[bake] = r.read_accum()
    print(json.dumps({"scene": name, **{"bake%d_ms" % k: round(float(np.median(v)), 2) for k, v in res.items()},
                      "bitwise_equal": bool(np.array_equal(img[0].view(np.uint32), img[1].view(np.uint32)))}), flush=True)
r.close()
