"""Launch-slot A/B (round 6): one context per variant (diagnostic library: RMR_LAUNCH_STREAMS and
RMR_SLOT_RESERVE read at scene load), rounds interleaved, three call patterns of the reference's loop at
1080p on a 4x4 tile grid, each ending in a sync:
    tiles  — one rmr_render_spp per tile (rmr_cli's batched loop: 16 launches per frame)
    frame  — one launch over the frame (nothing to overlap)
    calls  — rmr_render per tile and sample, call batching off (one launch per call)
Prints one JSON line per (config, pattern): median ms per frame per variant and bitwise equality.

    python tools/slot_ab.py [--cases rm3,c2] [--spp 4] VARIANT ...   (VARIANT = label=ls,reserve)"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["RMR_LIB"] = "diag"
import numpy as np  # noqa: E402
from raymarchrenderer_amd import Renderer, abi, tile_spiral, time_schedule  # noqa: E402

S, G = os.path.join(ROOT, "scenes"), os.path.join(ROOT, "tests", "golden", "scenes")
CASES = {"rm3": (None, "rm3", 16), "c2": (os.path.join(S, "cornell5.scene"), "rm1", 4),
         "rm2": (os.path.join(G, "simple.scene"), "rm2", 16)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--cases", default="rm3,c2")
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    W, H = 1920, 1080
    cw, ch = W // 4, H // 4
    rects = [((x * cw, y * ch), ((x + 1) * cw, (y + 1) * ch)) for x, y in tile_spiral(4, 4)]
    for name in a.cases.split(","):
        path, variant, bounces = CASES[name]
        times = time_schedule(a.spp)
        ctx = []
        for v in a.variants:
            label, _, spec = v.partition("=")
            ls, rs = (int(t) for t in spec.split(","))
            os.environ["RMR_LAUNCH_STREAMS"], os.environ["RMR_SLOT_RESERVE"] = str(ls), str(rs)
            r = Renderer(0, W, H)
            if path is None:
                r.load_builtin(variant)
            else:
                r.load_scene(path, variant)
            r.set_params(abi.default_params(max_bounces=bounces))
            ctx.append((label, r))
        for pat in ("tiles", "frame", "calls"):
            ms = {l: [] for l, _ in ctx}
            img = {}
            for rnd in range(a.rounds + 1):
                for label, r in ctx:
                    r.set_call_batching(0 if pat == "calls" else -1)
                    r.reload()
                    r.sync()
                    t0 = time.perf_counter()
                    if pat == "tiles":
                        for mn, mx in rects:
                            r.render_spp(times, rect=(mn[0], mn[1], mx[0], mx[1]))
                    elif pat == "frame":
                        r.render_spp(times, rect=(0, 0, cw * 4, ch * 4))
                    else:
                        for mn, mx in rects:
                            for s, t in enumerate(times):
                                r.render(float(t), mn, mx, s)
                    r.sync()
                    if rnd:
                        ms[label].append((time.perf_counter() - t0) * 1e3)
                    if rnd == a.rounds:
                        img[label] = r.read_accum()
            first = ctx[0][0]
            out = {"case": name, "pattern": pat, "spp": a.spp}
            for label, _ in ctx:
                out[label] = {"median_ms": round(float(np.median(ms[label])), 3),
                              "vs_first": round(float(np.median(ms[label]) / np.median(ms[first])), 4),
                              "bitwise_equal_to_first": bool(np.array_equal(img[label].view(np.uint32), img[first].view(np.uint32)))}
            print(json.dumps(out), flush=True)
        for _, r in ctx:
            r.close()


if __name__ == "__main__":
    main()
