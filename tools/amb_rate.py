"""Diagnostics: how often the approximate-then-exact map (rmr_trace.h am_*) falls back to the exact
fold, per scene (RMR_JIT_AMBCOUNT=1 build of the JIT source; raw counters [4], [5] via rmr_get_counters)."""
import ctypes as C
import json
import os
import sys

import numpy as np

os.environ["RMR_JIT_AMBCOUNT"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402

G = os.path.join(ROOT, "tests", "golden", "scenes")
r = Renderer(0, 1920, 1080)
r.set_jit(1)
for name, path, b in [("cornell5", os.path.join(ROOT, "scenes", "cornell5.scene"), 4),
                      ("multilight", os.path.join(G, "multilight.scene"), 16)]:
    r.load_scene(path, "rm1")
    r.set_params(abi.default_params(max_bounces=b))
    r.reload()
    r.reset_stats()
    r.render_spp(time_schedule(4))
    st = r.stats()
    raw = r.counters()
    out = [raw[4], raw[5]]
    cls = {"nan_point": raw[6], "exact_tie": raw[7], "near_surface": raw[9], "l2_tiny": raw[10]}
    f = lambda v: float(np.array([v & 0xffffffff], np.uint32).view(np.float32)[0])
    cls["sample_tie_point"] = [f(raw[11]), f(raw[12]), f(raw[13])]
    cls["sample_tie_dist_id"] = [f(raw[14]), f(raw[15])]
    print(json.dumps({"scene": name, "map_evals": st.map_evals, "map_iters": st.map_iters,
                      "amb_lanes": out[0], "amb_waves": out[1],
                      "amb_lane_frac": out[0] / max(1, st.map_evals), "amb_iter_frac": out[1] / max(1, st.map_iters),
                      "amb_lanes_by_class": cls}))
r.close()
