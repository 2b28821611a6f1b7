"""March / shade split diagnostics (rmr_trace.h trace_split): per schedule, trace time, lanes per
map() iteration and per shading batch; with --stats the kernel is built with -DRMR_SPLIT_STATS and
the shading wave's batch counts and cycle split and the marching waves' starved share are printed.

    python tools/split_stats.py [--scene cornell5] [--spp 16] [--stats] [--shade-t 6]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="cornell5")
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--W", type=int, default=1920)
ap.add_argument("--H", type=int, default=1080)
ap.add_argument("--bounces", type=int, default=4)
ap.add_argument("--stats", action="store_true")
ap.add_argument("--shade-t", default="", help="comma-separated shading thresholds to try (split)")
ap.add_argument("--opts", default="", help="extra RMR_JIT_OPTS")
a = ap.parse_args()
opts = (a.opts + (" -DRMR_SPLIT_STATS" if a.stats else "")).strip()
if opts:
    os.environ["RMR_JIT_OPTS"] = opts

import numpy as np  # noqa: E402
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402

path = None if a.scene == "rm3" else os.path.join(ROOT, "scenes", a.scene + ".scene")
r = Renderer(0, a.W, a.H)
r.set_jit(1)
times = time_schedule(a.spp)
img = {}
runs = [("mega", abi.SCHED_MEGA, 20)] + [("split", abi.SCHED_SPLIT, int(t)) for t in (a.shade_t.split(",") if a.shade_t else ["0"])]
for rnd in range(2):
    for name, sched, t in runs:
        r.set_schedule(sched)
        r.set_tuning(t if t else 0, -1, -1)
        if path is None:
            r.load_builtin("rm3")
        else:
            r.load_scene(path, "rm1")
        r.set_params(abi.default_params(max_bounces=a.bounces))
        r.reload()
        r.reset_stats()
        r.render_spp(times)
        st = r.stats()
        c = r.counters()
        img[(name, t)] = r.read_accum()
        if rnd == 0:
            continue
        out = {"sched": name, "shade_t": t, "trace_ms": round(st.trace_ms, 2), "maps": int(c[0]),
               "lanes_per_iter": round(c[0] / max(1, c[1]), 2), "batches": int(c[2]),
               "lanes_per_batch": round(c[8] / max(1, c[2]), 2)}
        if a.stats and sched == abi.SCHED_SPLIT:
            out.update({"hit_batches": int(c[4]), "fresh_batches": int(c[5]),
                        "shade_busy_hit": round(c[7] / max(1, c[6]), 3), "shade_busy_fresh": round(c[9] / max(1, c[6]), 3),
                        "march_starved": round(c[10] / max(1, c[15]), 3)})
        print(json.dumps(out), flush=True)
ref = img[("mega", 20)].view(np.uint32)
print(json.dumps({"bitwise_equal": all(np.array_equal(ref, v.view(np.uint32)) for v in img.values())}))
r.close()
