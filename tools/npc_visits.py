"""Nearest-primitive cache, full BVH batches (rmr_trace.h map_bvh_npc): per batch, the wave-level node
tests and primitive evaluations of the wave-uniform traversal against the largest per-lane need (the
cost a per-lane traversal would have). Kernel built with RMR_JIT_OPTS=-DRMR_NPC_VISITS.

    python tools/npc_visits.py [--spp 4]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
os.environ["RMR_JIT_OPTS"] = (os.environ.get("RMR_JIT_OPTS", "") + " -DRMR_NPC_VISITS").strip()
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
c = r.counters()
n = max(1, c[9])
print(json.dumps({"batches": c[9], "wave_node_tests": round(c[4] / n, 1), "wave_prim_evals": round(c[5] / n, 1),
                  "max_lane_node_tests_est": round(c[6] / n, 1), "max_lane_prims": round(c[7] / n, 1),
                  "lanes_per_batch": round(c[0] / max(1, c[1]), 1)}))
r.close()
