"""Where a persistent trace launch spends its fixed cost: per-wave start, queue-exhaustion and end
times (s_memrealtime, 100 MHz) from the RMR_WAVE_TIMES diagnostic build of the specialised kernel.
GPU only.   python tools/wave_times.py [--spp 8,64]"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
os.environ["RMR_JIT_OPTS"] = (os.environ.get("RMR_JIT_OPTS", "") + " -DRMR_WAVE_TIMES").strip()
from raymarchrenderer_amd import Renderer, abi, lib, time_schedule  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spp", default="8,64")
ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "cornell5.scene"))
ap.add_argument("--bounces", type=int, default=4)
ap.add_argument("--variant", default="rm1", help="rm1 / rm2 / rm3 (rm3: --scene builtin)")
ap.add_argument("--W", type=int, default=1920)
ap.add_argument("--H", type=int, default=1080)
a = ap.parse_args()
r = Renderer(0, a.W, a.H)
r.set_jit(1)
if a.scene == "builtin":
    r.load_builtin(a.variant)
else:
    r.load_scene(a.scene, a.variant)
r.set_params(abi.default_params(max_bounces=a.bounces))
r.reload()
r.render_spp(time_schedule(2))
M = (1 << 64) - 1
for s in [int(x) for x in a.spp.split(",")]:
    r.reset_stats()
    r.render_spp(time_schedule(s))
    r.sync()
    c = r.counters()
    st = r.stats()
    t0 = M ^ c[9]
    us = lambda t: round((t - t0) / 100.0, 1)   # 100 MHz ticks -> us after the first wave's start
    print(json.dumps({"spp": s, "trace_ms": round(st.trace_ms, 3), "launches": int(st.trace_launches),
                      "first_exhaust_us": us(M ^ c[11]), "last_exhaust_us": us(c[10]),
                      "first_end_us": us(M ^ c[12]), "last_end_us": us(c[13]),
                      "mean_drain_us": round(c[15] / 100.0 / max(1, 8192), 1), "label": "%s %dx%d" % (
                          os.path.basename(a.scene), a.W, a.H)}), flush=True)
r.close()
