"""Same-process A/B runner: every measured experiment of rounds 1-4 (library builds, compile-time
switches, environment switches, culling flags, tuning) in one tool with one config table.

    python tools/abrun.py [--cases c2,rm3] [--spp N] [--rounds R] VARIANT [VARIANT ...]

VARIANT = [LABEL=]SPEC[;SPEC...], SPEC one of
    lib:PATH        the context lives in that librmr build (default: the diagnostic library, which
                    reads the RMR_* switches; e.g. tools/build_rev.sh HEAD tools/librmr_base.so)
    opts:WORDS      RMR_JIT_OPTS (hipRTC compiler options, e.g. -DRMR_PROG_WAVES=6)
    env:K=V         any other RMR_* switch read at scene load / specialisation time (repeatable)
    cull:N          rmr_set_culling flags
    shade:T         rmr_set_tuning shading threshold (T + 256 R: refill threshold R)
e.g.  python tools/abrun.py --cases c2,c4 base="lib:tools/librmr_base.so" new="lib:raymarchrenderer_amd/librmr_diag.so"
      python tools/abrun.py --cases glass,default w6="opts:-DRMR_PROG_WAVES=6" w7="opts:-DRMR_PROG_WAVES=7" def=""

Each variant has its own context; rounds alternate between the variants (MI355X_MICROARCH rule 24:
compare in one process, interleaved), round 0 is warm-up (hipRTC compile). Per case one JSON line:
median / min trace-kernel ms per variant, the ratio to the first variant, the kernel counters, and
whether the accumulator is bitwise equal to the first variant's.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np  # noqa: E402
from raymarchrenderer_amd import Renderer, abi, time_schedule  # noqa: E402

S, G = os.path.join(ROOT, "scenes"), os.path.join(ROOT, "tests", "golden", "scenes")
# name: scene file (None: the built-in RM3 scene), variant, bounces, W, H, default spp
CASES = {
    "c1": (os.path.join(S, "sphere1.scene"), "rm1", 1, 256, 256, 1),
    "c2": (os.path.join(S, "cornell5.scene"), "rm1", 4, 1920, 1080, 16),
    "c3": (os.path.join(S, "mandelbulb.scene"), "rm1", 2, 1920, 1080, 16),
    "c4": (os.path.join(S, "csg256.scene"), "rm1", 4, 1920, 1080, 8),
    "rm2": (os.path.join(G, "simple.scene"), "rm2", 16, 1920, 1080, 16),
    "rm3": (None, "rm3", 16, 1920, 1080, 16),
    "glass": (os.path.join(G, "glass_test.scene"), "rm1", 16, 1920, 1080, 16),
    "default": (os.path.join(G, "default.scene"), "rm1", 16, 1920, 1080, 16),
    "multilight": (os.path.join(G, "multilight.scene"), "rm1", 16, 1920, 1080, 16),
    "csg64": (os.path.join(S, "csg64.scene"), "rm1", 4, 1920, 1080, 8),
    "csg_nodes": (os.path.join(S, "csg_nodes.scene"), "rm1", 4, 1920, 1080, 8),
    # one tile of the reference's 4x4 grid at 1080p, one sample: a Graphics::Render call's launch
    "c2t": (os.path.join(S, "cornell5.scene"), "rm1", 4, 480, 270, 1),
    "rm3t": (None, "rm3", 16, 480, 270, 1),
    "c3t": (os.path.join(S, "mandelbulb.scene"), "rm1", 2, 480, 270, 1),
}


def parse_variant(text):
    label, _, spec = text.partition("=") if ("=" in text.split(":")[0]) else ("", "", text)
    v = {"label": label or text or "default", "lib": None, "env": {}, "cull": None, "shade": None}
    for item in filter(None, spec.split(";")):
        kind, _, val = item.partition(":")
        if kind == "lib":
            v["lib"] = val
        elif kind == "opts":
            v["env"]["RMR_JIT_OPTS"] = val
        elif kind == "env":
            k, _, x = val.partition("=")
            v["env"][k] = x
        elif kind == "cull":
            v["cull"] = int(val)
        elif kind == "shade":
            v["shade"] = int(val)
        else:
            raise SystemExit("unknown variant spec %r" % item)
    return v


def apply_env(v, keys, saved):
    for k in keys:
        if k in v["env"]:
            os.environ[k] = v["env"][k]
        elif saved.get(k) is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = saved[k]


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--cases", default="c2")
    ap.add_argument("--spp", type=int, default=0, help="samples per pixel (0: the case's default)")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--W", type=int, default=0)
    ap.add_argument("--H", type=int, default=0)
    ap.add_argument("--raw", action="store_true", help="also print the 16 raw kernel counters (diagnostic builds)")
    a = ap.parse_args()
    vs = [parse_variant(t) for t in a.variants]
    keys = sorted({k for v in vs for k in v["env"]})
    saved = {k: os.environ.get(k) for k in keys}
    ctx = [Renderer(0, 64, 64, diag=(v["lib"] if v["lib"] else True)) for v in vs]
    for name in a.cases.split(","):
        path, variant, bounces, W, H, spp = CASES[name]
        W, H, spp = a.W or W, a.H or H, a.spp or spp
        times = time_schedule(spp)
        ms = [[] for _ in vs]
        img, st, cnt = [None] * len(vs), [None] * len(vs), [None] * len(vs)
        for rnd in range(a.rounds + 1):
            for i, (v, r) in enumerate(zip(vs, ctx)):
                apply_env(v, keys, saved)
                r.set_image_size(W, H)
                r.set_jit(1)
                if path is None:
                    r.load_builtin(variant)
                else:
                    r.load_scene(path, variant)
                r.set_params(abi.default_params(max_bounces=bounces))
                if v["cull"] is not None:
                    r.set_culling(v["cull"])
                if v["shade"] is not None:
                    r.set_tuning(v["shade"], -1, 0)
                r.reload()
                r.reset_stats()
                r.render_spp(times)
                s = r.stats()
                if rnd:
                    ms[i].append(s.trace_ms)
                if rnd == a.rounds:
                    img[i], st[i], cnt[i] = r.read_accum(), s, r.counters()
        apply_env({"env": {}}, keys, saved)
        t0 = float(np.median(ms[0]))
        out = {"case": name, "W": W, "H": H, "spp": spp, "bounces": bounces}
        for i, v in enumerate(vs):
            t = np.array(ms[i])
            out[v["label"]] = {
                "median_ms": round(float(np.median(t)), 3), "min_ms": round(float(t.min()), 3),
                "vs_first": round(float(np.median(t)) / t0, 4),
                "Msamples_s": round(W * H * spp / float(np.median(t)) / 1e3, 1),
                "map_evals": int(st[i].map_evals), "map_iters": int(st[i].map_iters),
                "shade_batches": int(st[i].shade_batches),
                "lanes_per_batch": round(cnt[i][8] / max(1, st[i].shade_batches), 2),
                "bitwise_equal_to_first": bool(np.array_equal(img[i].view(np.uint32), img[0].view(np.uint32))),
            }
            if a.raw:
                out[v["label"]]["raw"] = cnt[i]
            if "-DRMR_PROFILE" in v["env"].get("RMR_JIT_OPTS", ""):
                # section cycles of the profiling build (rmr_trace.h RMR_PROFILE: counters 4-7, 9),
                # as fractions of the waves' cycles (the s_memtime stamps themselves cost ~10%)
                c, tot = cnt[i], max(1, cnt[i][7])
                out[v["label"]]["sections"] = {"refill": round(c[4] / tot, 4), "map_loop": round(c[5] / tot, 4),
                                               "shade": round(c[6] / tot, 4), "cache_full_maps": round(c[9] / tot, 4),
                                               # parts of refill: work-queue claims, the chunk's primary rays
                                               "refill_claims": round(c[11] / tot, 4), "refill_rays": round(c[12] / tot, 4)}
                if c[3]:   # cache kernels: lanes per full map() batch (counter 10 of the profiling build)
                    out[v["label"]]["lanes_per_full_batch"] = round(c[10] / c[3], 2)
        print(json.dumps(out), flush=True)
    for r in ctx:
        r.close()


if __name__ == "__main__":
    main()
