"""One C2 render (1080p, --spp) with the current environment; prints the kernel counters as JSON
(map evals, map iterations, shading batches, trace ms). Run under rocprofv3 --pmc for per-launch
instruction counts (tools/pmc_sweep.sh)."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "cornell5.scene"))
ap.add_argument("--bounces", type=int, default=4)
ap.add_argument("--variant", default="rm1", help="rm1 / rm2 / rm3 (rm3: --scene builtin)")
a = ap.parse_args()
r = Renderer(0, 1920, 1080)
r.set_jit(1)
if a.scene == "builtin":
    r.load_builtin(a.variant)
else:
    r.load_scene(a.scene, a.variant)
r.set_params(abi.default_params(max_bounces=a.bounces))
r.reload()
r.render_spp(time_schedule(a.spp))   # warm-up (JIT compile)
r.reset_stats()
r.render_spp(time_schedule(a.spp))
st = r.stats()
raw = r.counters()
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("RMR_")}, "trace_ms": round(st.trace_ms, 3),
                  "map_evals": st.map_evals, "map_iters": st.map_iters, "shade_batches": st.shade_batches,
                  "lanes_shaded": raw[8], "lanes_per_batch": round(raw[8] / max(1, st.shade_batches), 2),
                  "evals_per_iter": round(st.map_evals / max(1, st.map_iters), 2),
                  "raw": [int(v) for v in raw]}))
r.close()
