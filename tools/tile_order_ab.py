import os, sys, json
sys.path.insert(0, "/root/repo")
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np
from raymarchrenderer_amd import Renderer, abi, time_schedule
from raymarchrenderer_amd.multi_gpu import tile_partition
r = Renderer(0, 1920, 1080)
r.load_scene("/root/repo/scenes/cornell5.scene", "rm1")
r.set_params(abi.default_params(max_bounces=4))
times = time_schedule(64)
tiles = tile_partition(1920, 1080, 32, 0, 1)
res = {"rect": [], "tiles32": [], "tiles8": []}
t8 = tile_partition(1920, 1080, 8, 0, 1)
for rnd in range(4):
    for k in res:
        r.reload(); r.reset_stats()
        if k == "rect": r.render_spp(times)
        elif k == "tiles32": r.render_tiles(times, tiles, 32)
        else: r.render_tiles(times, t8, 8)
        st = r.stats()
        if rnd: res[k].append(st.trace_ms)
print(json.dumps({k: round(float(np.median(v)), 3) for k, v in res.items()}))
