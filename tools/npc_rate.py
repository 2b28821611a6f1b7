"""Diagnostics of the nearest-primitive cache (rmr_trace.h npc_*): fraction of map() evaluations
served by one cached primitive vs full BVH batches, per full_threshold (RMR_FULL_T)."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402

r = Renderer(0, 1920, 1080)
r.set_jit(1)
r.load_scene(os.path.join(ROOT, "scenes", "csg256.scene"), "rm1")
r.set_params(abi.default_params(max_bounces=4))
r.reload()
for rnd in range(2):
    r.reset_stats()
    r.render_spp(time_schedule(4))
    st = r.stats()
raw = r.counters()
print(json.dumps({"full_threshold": os.environ.get("RMR_FULL_T", "default"), "trace_ms": round(st.trace_ms, 2),
                  "map_evals": st.map_evals, "map_iters": st.map_iters, "full_batches": raw[3],
                  "lane_util": round(st.map_evals / (64.0 * st.map_iters), 4),
                  "full_batches_per_iter": round(raw[3] / st.map_iters, 4),
                  # with RMR_JIT_OPTS=-DRMR_NPC_AMBCOUNT: lanes / batches that took the exact traversal
                  "exact_fallback_lanes": raw[9], "exact_fallback_batches": raw[10]}))
r.close()
