"""Does the launch's tail depend on which pixels run last? C2 at --spp, the same 32x32 tile list in
raster order, reversed, and bottom-half-first; trace time per order and a bitwise check (tile order
changes only scheduling)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np  # noqa: E402
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402
from raymarchrenderer_amd.multi_gpu import tile_partition  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=8)
ap.add_argument("--rounds", type=int, default=4)
a = ap.parse_args()
r = Renderer(0, 1920, 1080)
r.set_jit(1)
r.load_scene(os.path.join(ROOT, "scenes", "cornell5.scene"), "rm1")
r.set_params(abi.default_params(max_bounces=4))
times = time_schedule(a.spp)
base = np.asarray(tile_partition(1920, 1080, 32, 0, 1))
orders = {"raster": base, "reversed": base[::-1].copy(),
          "bottom_first": np.concatenate([base[base[:, 1] >= 540], base[base[:, 1] < 540]])}
res, img = {}, {}
for rnd in range(a.rounds + 1):
    for k, t in orders.items():
        r.reload()
        r.reset_stats()
        r.render_tiles(times, t, 32)
        if rnd:
            res.setdefault(k, []).append(r.stats().trace_ms)
        img[k] = r.read_accum().view(np.uint32).copy()
print(json.dumps({**{k: round(float(np.median(v)), 3) for k, v in res.items()},
                  "bitwise_equal": all(np.array_equal(img["raster"], v) for v in img.values())}))
r.close()
