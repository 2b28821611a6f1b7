"""Candidate-grid diagnostics of the nearest-primitive cache's full map() batches (rmr_trace.h
map_grid_npc, kernel built with RMR_JIT_OPTS=-DRMR_GRID_STATS): batches, lanes per batch, listed
primitives per lane, longest list per batch, lanes outside the grid (BVH path).

    python tools/grid_stats.py [--spp 4] [--scene scenes/csg256.scene]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
os.environ["RMR_JIT_OPTS"] = (os.environ.get("RMR_JIT_OPTS", "") + " -DRMR_GRID_STATS").strip()
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=4)
ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "csg256.scene"))
a = ap.parse_args()
r = Renderer(0, 1920, 1080)
r.set_jit(1)
r.load_scene(a.scene, "rm1")
r.set_params(abi.default_params(max_bounces=4))
r.reload()
r.reset_stats()
r.render_spp(time_schedule(a.spp))
st = r.stats()
c = r.counters()
nb = max(1, c[4])
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("RMR_")}, "trace_ms": round(st.trace_ms, 2),
                  "map_iters": st.map_iters, "full_batches": c[3], "grid_batches": c[4],
                  "lanes_per_grid_batch": round(c[7] / nb, 2), "listed_per_lane": round(c[6] / max(1, c[7]), 2),
                  "longest_list_per_batch": round(c[5] / nb, 2), "lanes_taking_bvh": c[9], "lanes_outside_no_list": c[12],
                  "batches_with_bvh_part": c[10]}))
r.close()
