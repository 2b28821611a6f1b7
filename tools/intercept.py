"""Per-launch fixed cost of the trace kernel: one process renders C2 (1080p) at several spp per
launch, interleaved rounds, and fits trace ms = a + b spp (least squares on the medians).
GPU only.   python tools/intercept.py [--spp 2,4,8,16,32,64] [--rounds 5]"""
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
ap.add_argument("--spp", default="2,4,8,16,32,64")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "cornell5.scene"))
ap.add_argument("--bounces", type=int, default=4)
a = ap.parse_args()
spps = [int(s) for s in a.spp.split(",")]
r = Renderer(0, 1920, 1080)
r.set_jit(1)
r.load_scene(a.scene, "rm1")
r.set_params(abi.default_params(max_bounces=a.bounces))
r.reload()
r.render_spp(time_schedule(2))   # JIT compile
res = {s: [] for s in spps}
for rnd in range(a.rounds):
    for s in spps:
        r.reset_stats()
        r.render_spp(time_schedule(s))
        res[s].append(r.stats().trace_ms)
med = np.array([np.median(res[s]) for s in spps])
x = np.array(spps, float)
b, c = np.polyfit(x, med, 1)
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("RMR_")},
                  "ms": {str(s): round(float(m), 3) for s, m in zip(spps, med)},
                  "slope_ms_per_spp": round(float(b), 4), "intercept_ms": round(float(c), 3)}))
r.close()
