"""A/B timing of librmr builds in ONE process (interleaved rounds, MI355X_MICROARCH rule 24).

    python tools/ab.py raymarchrenderer_amd/librmr.so raymarchrenderer_amd/librmr_x.so [...]

Each library gets its own rmr context; rounds alternate between them; reports median/min
trace-kernel ms per library on the C2 workload at reduced spp.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RMR_LIB", "diag")   # tools run against the diagnostic build (env switches)
import numpy as np  # noqa: E402
from raymarchrenderer_amd import abi, time_schedule  # noqa: E402


def load(path):
    L = C.CDLL(os.path.abspath(path))
    vp = C.c_void_p
    fp = C.POINTER(C.c_float)
    L.rmr_create.argtypes = [C.POINTER(vp), C.c_int]
    L.rmr_set_image_size.argtypes = [vp, C.c_int, C.c_int]
    L.rmr_reload.argtypes = [vp]
    L.rmr_load_scene_json.argtypes = [vp, C.c_int, C.c_char_p, C.c_size_t]
    L.rmr_load_builtin_scene.argtypes = [vp, C.c_int]
    L.rmr_set_params.argtypes = [vp, C.POINTER(abi.Params)]
    L.rmr_render_spp.argtypes = [vp, fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_uint32]
    L.rmr_get_stats.argtypes = [vp, C.POINTER(abi.Stats)]
    L.rmr_reset_stats.argtypes = [vp]
    L.rmr_set_tuning.argtypes = [vp, C.c_int, C.c_int, C.c_longlong]
    L.rmr_read_accum.argtypes = [vp, fp, C.c_size_t]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "cornell5.scene"))
    ap.add_argument("--variant", type=int, default=1)
    ap.add_argument("--bounces", type=int, default=4)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--T", type=int, default=0)
    args = ap.parse_args()
    text = open(args.scene).read().encode() if args.scene != "builtin" else b""
    ctxs = []
    for spec in args.libs:
        # "path.so" or "path.so:FLAGS" (rmr_set_culling flags for this context)
        p, _, cf = spec.partition(":")
        L = load(p)
        h = C.c_void_p()
        assert L.rmr_create(C.byref(h), 0) == 0
        L.rmr_set_image_size(h, args.W, args.H)
        L.rmr_reload(h)
        if text:
            assert L.rmr_load_scene_json(h, args.variant, text, len(text)) == 0
        else:
            assert L.rmr_load_builtin_scene(h, args.variant) == 0
        prm = abi.default_params(max_bounces=args.bounces)
        L.rmr_set_params(h, C.byref(prm))
        if args.T:
            L.rmr_set_tuning(h, args.T, -1, 0)
        if cf:
            L.rmr_set_culling.argtypes = [C.c_void_p, C.c_int]
            assert L.rmr_set_culling(h, int(cf)) == 0
        ctxs.append((spec, L, h))
    times = time_schedule(args.spp)
    tp = times.ctypes.data_as(C.POINTER(C.c_float))
    res = {p: [] for p, _, _ in ctxs}
    stats = {}
    imgs = {}
    for rnd in range(args.rounds + 1):
        for p, L, h in ctxs:
            L.rmr_reset_stats(h)
            L.rmr_render_spp(h, tp, 0, 0, args.W, args.H, 0, args.spp)
            st = abi.Stats()
            L.rmr_get_stats(h, C.byref(st))
            if rnd > 0:
                res[p].append(st.trace_ms)
            stats[p] = st
            if rnd == args.rounds and hasattr(L, "rmr_get_section_cycles"):
                cy = (C.c_uint64 * 4)()
                L.rmr_get_section_cycles(h, cy)
                if cy[3]:
                    print(json.dumps({"lib": os.path.basename(p), "cycles_refill": cy[0] / cy[3],
                                      "cycles_map": cy[1] / cy[3], "cycles_shade": cy[2] / cy[3],
                                      "lane_util": st.map_evals / (64.0 * max(1, st.map_iters)),
                                      "maps_per_iter_batch": st.map_iters / max(1, st.shade_batches)}), flush=True)
            if rnd == args.rounds:
                a = np.zeros((args.H, args.W, 4), np.float32)
                L.rmr_read_accum(h, a.ctypes.data_as(C.POINTER(C.c_float)), a.nbytes)
                imgs[p] = a
    base = args.libs[0]
    for p in args.libs:
        t = np.array(res[p])
        same = np.array_equal(imgs[p].view(np.uint32), imgs[base].view(np.uint32))
        st = stats[p]
        print(json.dumps({"lib": os.path.basename(p), "median_ms": round(float(np.median(t)), 3),
                          "min_ms": round(float(t.min()), 3),
                          "Msamples/s": round(args.W * args.H * args.spp / np.median(t) / 1e3, 1),
                          "map_evals": int(st.map_evals), "map_iters": int(st.map_iters),
                          "shade_batches": int(st.shade_batches),
                          "bitwise_equal_to_first": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
