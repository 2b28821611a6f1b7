"""Trace-kernel time, table-driven vs hipRTC-specialised, per scene (same process, interleaved).
GPU only.   python tools/jit_ab.py [--W 1920 --H 1080 --spp 16]"""
import argparse
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
         ("glass_test", os.path.join(G, "glass_test.scene"), "rm1", 16),
         ("multilight", os.path.join(G, "multilight.scene"), "rm1", 16),
         ("simple_rm2", os.path.join(G, "simple.scene"), "rm2", 16), ("rm3", None, "rm3", 16),
         ("mandelbulb", os.path.join(S, "mandelbulb.scene"), "rm1", 2), ("csg256", os.path.join(S, "csg256.scene"), "rm1", 4)]
ap = argparse.ArgumentParser()
ap.add_argument("--W", type=int, default=1920)
ap.add_argument("--H", type=int, default=1080)
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--rounds", type=int, default=3)
args = ap.parse_args()
r = Renderer(0, args.W, args.H)
times = time_schedule(args.spp)
for name, path, var, b in CASES:
    if path is None:
        r.load_builtin(var)
    else:
        r.load_scene(path, var)
    r.set_params(abi.default_params(max_bounces=b))
    res = {0: [], 1: []}
    img = {}
    for rnd in range(args.rounds + 1):
        for mode in (0, 1):
            r.set_jit(mode)
            r.reload()
            r.reset_stats()
            r.render_spp(times)
            st = r.stats()
            if rnd:
                res[mode].append(st.trace_ms)
            img[mode] = r.read_accum()
    same = np.array_equal(img[0].view(np.uint32), img[1].view(np.uint32))
    t0, t1 = float(np.median(res[0])), float(np.median(res[1]))
    print(json.dumps({"scene": name, "table_ms": round(t0, 2), "jit_ms": round(t1, 2), "speedup": round(t0 / t1, 3),
                      "jit_Msamples/s": round(args.W * args.H * args.spp / t1 / 1e3, 1), "bitwise_equal": same}),
          flush=True)
r.close()
