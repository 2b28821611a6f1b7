"""Parameter sweep of the trace kernel on the C2 workload (reduced spp). GPU only."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np  # noqa: E402
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "cornell5.scene"))
ap.add_argument("--variant", default="rm1")
ap.add_argument("--bounces", type=int, default=4)
ap.add_argument("--W", type=int, default=1920)
ap.add_argument("--H", type=int, default=1080)
ap.add_argument("--configs", default="")
args = ap.parse_args()

r = Renderer(0, args.W, args.H)
if args.scene == "builtin":
    r.load_builtin(args.variant)
else:
    r.load_scene(args.scene, args.variant)
r.set_params(abi.default_params(max_bounces=args.bounces))
times = time_schedule(args.spp)
configs = json.loads(args.configs) if args.configs else [
    {"kernel": 1}, {"kernel": 0, "T": 1}, {"kernel": 0, "T": 8}, {"kernel": 0, "T": 16},
    {"kernel": 0, "T": 24}, {"kernel": 0, "T": 32}, {"kernel": 0, "T": 48}, {"kernel": 0, "T": 64},
    {"kernel": 0, "T": 24, "grid": 2}, {"kernel": 0, "T": 24, "grid": 8}]
for cfg in configs:
    r.set_kernel(cfg.get("kernel", 0))
    r.set_tuning(shade_threshold=cfg.get("T", 24) | (cfg.get("TR", 0) << 8), grid_per_cu=cfg.get("grid", 0))
    r.render_spp(times[:2])
    r.sync()
    r.reset_stats()
    t0 = time.perf_counter()
    r.render_spp(times)
    r.sync()
    dt = time.perf_counter() - t0
    st = r.stats()
    util = st.map_evals / max(1, 64 * st.map_iters)
    print(json.dumps({"cfg": cfg, "Msamples/s": round(args.W * args.H * args.spp / dt / 1e6, 1),
                      "trace_ms": round(st.trace_ms, 2), "maps/sample": round(st.map_evals / (args.W * args.H * args.spp), 2),
                      "lane_util": round(util, 3), "Gmaps/s": round(st.map_evals / (st.trace_ms * 1e-3) / 1e9, 2),
                      "shade_batches/iter": round(st.shade_batches / max(1, st.map_iters), 3)}), flush=True)
r.close()
