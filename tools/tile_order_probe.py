"""Does the order of a frame's tiles change the trace launch's time? The work queue hands units out in
tile-list order within each sample, so the launch's last units (its drain) are the last tiles of the
last sample. Same frame, same bits, 32x32 tiles (the frame renderer's) in row-major, reversed and
shuffled order, and sorted by cost: each tile's map() evaluations in a 2-sample probe, costliest first
(multi_gpu.FrameRenderer.order_tiles_by_cost). GPU only.
    python tools/tile_order_probe.py [--cases c2,c3] [--spp 16] [--rounds 5]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402
from raymarchrenderer_amd.multi_gpu import tile_costs  # noqa: E402

S = os.path.join(ROOT, "scenes")
CASES = {"c2": ("cornell5.scene", 4), "c3": ("mandelbulb.scene", 2), "c4": ("csg256.scene", 4)}

ap = argparse.ArgumentParser()
ap.add_argument("--cases", default="c2,c3")
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--rounds", type=int, default=5)
a = ap.parse_args()
W, H, TS = 1920, 1080, 32
tiles = np.array([(x, y) for y in range((H + TS - 1) // TS) for x in range((W + TS - 1) // TS)], np.int32)   # tile indices
rng = np.random.default_rng(3)
r = Renderer(0, W, H)
r.set_jit(1)
for name in a.cases.split(","):
    scene, bounces = CASES[name]
    r.load_scene(os.path.join(S, scene), "rm1")
    r.set_params(abi.default_params(max_bounces=bounces))
    r.reload()
    times = time_schedule(a.spp)
    cost = tile_costs(r, tiles, TS, time_schedule(2))
    orders = {"rows": tiles, "rows_reversed": tiles[::-1].copy(), "shuffled": tiles[rng.permutation(len(tiles))],
              "cost_sorted": tiles[np.argsort(-cost, kind="stable")]}
    ms = {k: [] for k in orders}
    img = {}
    for rnd in range(a.rounds + 1):
        for k, t in orders.items():
            r.reload()
            r.reset_stats()
            r.render_tiles(times, t, TS)
            st = r.stats()
            if rnd:
                ms[k].append(st.trace_ms)
            if rnd == a.rounds:
                img[k] = r.read_accum()
    base = float(np.median(ms["rows"]))
    print(json.dumps({"case": name, "spp": a.spp, "tile_cost_max_over_mean": round(float(cost.max() / cost.mean()), 2),
                      **{k: {"median_ms": round(float(np.median(v)), 3), "vs_rows": round(float(np.median(v)) / base, 4),
                             "bitwise_equal_to_rows": bool(np.array_equal(img[k].view(np.uint32), img["rows"].view(np.uint32)))}
                         for k, v in ms.items()}}), flush=True)
r.close()
