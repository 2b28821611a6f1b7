"""bench.py — headline benchmark: Msamples/s (pixels x spp) of the SDF ray-march path tracer.

Default workload (BASELINE.json configs[1]): Cornell-5 SDF scene
(scenes/cornell5.scene, RayMarch.glsl semantics), 1920x1080, 64 spp, 4 bounces, default camera
(Program.cpp:102), seed schedule time(f, s) = 1000 f + 0.016 s. One step = one full frame: every
pixel's spp samples traced, folded into the RGBA32F running mean, and (N > 1) the per-rank tile
accumulators summed onto rank 0 by one RCCL reduce.

The other BASELINE configs run with --config (they are separate bench lines, not the headline):
  c1  single sphere 256x256, 1 spp, 1 bounce
  c3  Mandelbulb (scenes/mandelbulb.scene) 1920x1080, 128 spp, 2 bounces
  c4  256-prim union (scenes/csg256.scene) 3840x2160, 256 spp, 4 bounces
  c5  animated Cornell-5, 1920x1080, 512 spp, 4 bounces: step f renders frame f (sphere centre
      y = 0.5 sin(2 pi f / 120)); the scene is recompiled and uploaded inside the timed step
  rm3 RayMarch3.glsl as the reference wires it (Graphics.cpp:272): built-in spectral scene,
      1920x1080, 4 spp, 16 bounces (the reference's own CPU path measured 5.2-5.4 Msamples/s)
  rm2 RayMarch2.glsl (NEE) on simple.scene, 1920x1080, 4 spp, 16 bounces (llvmpipe 18-20)

Multi-GPU: one process per GPU (torch.distributed, backend nccl = RCCL). `--gpus N` without a
launcher's WORLD_SIZE starts N rank processes itself (before anything in the parent touches the
GPU); under `torch.distributed.run` the launcher's ranks are used. The frame's 32x32 tiles are dealt
round-robin to the ranks; each rank renders its tiles into a zeroed full-frame accumulator
(x + 0 = x, so the reduce is exact); frame f's reduce overlaps frame f + 1's render (two
accumulators), and with N > 1 consecutive frames also overlap on two HIP streams (two renderer
contexts), so one frame's persistent-kernel drain is filled by the next. Total work per step is
fixed => "scaling": "strong". Rank 0's line carries the per-rank trace times and the cost of one
frame reduce measured on its own (`multi_gpu`).

`--dry-run` runs the same multi-rank schedule on the CPU (gloo, the CPU oracle as each rank's
renderer, a 64x48 frame): rank 0 reports whether the reduced frame equals a one-process render bit
for bit (tests/test_bench_cpu.py). It measures nothing.

Prints ONE JSON line on rank 0 (see DESIGN.md §6 for every field).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Hardware queues per process (HIP's GPU_MAX_HW_QUEUES, default 4; the GPU box exports 4), raised to 8
# before anything initialises HIP: the frame path's overlapping contexts each need their stream on a
# queue of its own, and with 4 the third context's stream (or RCCL's) shares one and serialises behind
# another context's trace (C1 856 against 1,637 Msamples/s with three contexts; r06za_hwq.log). A
# caller's value of 8 or more is kept.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

METRIC = "Msamples/sec (pixels×spp) at 1920×1080; PSNR vs GLSL reference"
TILE = 32
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: peak FP32 vector (spec)
# measured on the box by tools/probes/fma_peak.hip (8 independent FMA chains per lane, 8 waves/SIMD):
# scalar v_fma_f32 and packed v_pk_fma_f32 (the spec figure counts the packed form)
FP32_MEASURED_TFLOPS = {"v_fma_f32": 73.8, "v_pk_fma_f32": 143.0}
# transcendental issue limit (v_sqrt / v_exp / v_log / v_rcp ...): 8 cycles per wave64 instruction on a
# SIMD against 4 for v_fma_f32 (MI355X_MICROARCH.md, "vector-instruction ISSUE cost"):
# 1024 SIMDs x 64 lanes / 8 cycles x 2.4 GHz
TRANSC_PEAK_PER_S = 1024 * 64 / 8 * 2.4e9

CONFIGS = {
    "c1": dict(scene="sphere1.scene", W=256, H=256, spp=1, bounces=1, name="C1 single-sphere SDF"),
    "c2": dict(scene="cornell5.scene", W=1920, H=1080, spp=64, bounces=4, name="C2 Cornell-5 SDF"),
    "c3": dict(scene="mandelbulb.scene", W=1920, H=1080, spp=128, bounces=2, name="C3 Mandelbulb SDF"),
    "c4": dict(scene="csg256.scene", W=3840, H=2160, spp=256, bounces=4, name="C4 256-prim CSG union"),
    "c5": dict(scene="cornell5.scene", W=1920, H=1080, spp=512, bounces=4, name="C5 animated Cornell-5",
               animated=True),
    # the reference's own kernels where its CPU path was measured: RayMarch3.glsl as
    # Graphics.cpp:272 wires it (3-primitive spectral scene, maxBounces 16) and the RM2 NEE variant on
    # simple.scene; 1920x1080, 4 spp, as measured on llvmpipe
    "rm3": dict(scene=None, variant="rm3", W=1920, H=1080, spp=4, bounces=16,
                name="RM3 as wired (RayMarch3.glsl built-in scene)"),
    "rm2": dict(scene="../tests/golden/scenes/simple.scene", variant="rm2", W=1920, H=1080, spp=4, bounces=16,
                name="RM2 simple.scene (RayMarch2.glsl NEE)"),
}


def variant_of(cfg):
    return cfg.get("variant", "rm1")


def load_into(r, cfg, scene):
    """Load a config's scene (path or dict; None = the variant's built-in scene) into a Renderer."""
    if scene is None:
        r.load_builtin(variant_of(cfg))
    else:
        r.load_scene(scene, variant_of(cfg))


def oracle_tables(cfg, scene):
    from oracle import scene_compile
    if scene is None:
        return scene_compile.compile_scene({}, variant_of(cfg))
    if isinstance(scene, str):
        return scene_compile.load_scene_file(scene, variant_of(cfg))
    return scene_compile.compile_scene(scene, variant_of(cfg))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override the config's spp")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-psnr", action="store_true", help="skip the converged PSNR check vs the reference render")
    ap.add_argument("--no-count-pass", action="store_true",
                    help="skip the executed-work count pass (roofline flops then use the static per-map count)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--kernel", type=int, default=0, help="0 persistent, 1 per-path")
    ap.add_argument("--shade-threshold", type=int, default=0)
    ap.add_argument("--traffic-json", default="")
    ap.add_argument("--overlap", type=int, default=-1,
                    help="K >= 1: K + 1 renderer contexts on as many streams, consecutive frames overlap on the GPU; "
                         "0: one context; default 3 (four contexts) where a rank's frame share is <= 20 M samples, "
                         "else 1 (two contexts: at N = 1 +1.3%% C2, +25%% RM3, +18%% RM2, +97%% C1, round 3; "
                         "default_overlap). The roofline's per-launch time then comes from "
                         "`steps` frames rendered one at a time after the timed region")
    ap.add_argument("--grid-reserve", type=int, default=-1,
                    help="with overlapping contexts, workgroups each trace launch leaves free for the other "
                         "context's fold (rmr_set_grid_reserve); default multi_gpu.OVERLAP_GRID_RESERVE")
    ap.add_argument("--tile-order", choices=["cost", "rows", "cost-always"], default="cost",
                    help="cost: where a rank's 32x32 tiles' costs are uneven (a 2-sample probe of every tile's map() "
                         "evaluations), trial frames in row and cost order before the timed region decide "
                         "(FrameRenderer.order_tiles_by_cost: costliest first, the launches' drains end on cheap "
                         "tiles; C3 +2.7%%, RM2 kept in rows, the others under the spread; same image bits); "
                         "rows: row-major; cost-always: cost order whatever the spread, no trial (experiments)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the multi-rank path (gloo + CPU oracle renderer); no GPU")
    ap.add_argument("--share-gpu", action="store_true",
                    help="GPU rehearsal of the multi-rank path on a one-GPU box: every rank renders on "
                         "cuda:0 with the HIP kernels, the frame reduce runs over gloo (staged through "
                         "host memory); a correctness rehearsal, not a scaling measurement")
    ap.add_argument("--predict", default="",
                    help="comma-separated rank counts (e.g. 2,4,8): on ONE GPU, time each rank's tile share of the "
                         "frame in turn (two overlapping contexts, as at N > 1) for 32x32 and 64x64 tiles, and the "
                         "sample-split alternative; prints the per-rank times, the imbalance and the predicted "
                         "speed-up (SURVEY §8e)")
    ap.add_argument("--no-verify", action="store_true",
                    help="N > 1: skip rank 0's check of the last reduced frame against a one-context render")
    ap.add_argument("--api", choices=["frame", "render", "group"], default="frame",
                    help="frame: the batched frame path (rmr_render_tiles, the headline); render: the reference's "
                         "own call pattern through the drop-in, Program.cpp:232-284's fixed-spp loop: a 4x4 tile "
                         "grid in spiral order, every tile's samples one rmr_render (Graphics::Render) call each, "
                         "no sync per call; one step = one frame (a separate line, not the headline); group: the "
                         "C++ host's single-process device group (librmr_group.so: --gpus N devices from ONE "
                         "process, ncclCommInitAll, one RCCL reduce per frame; not under a launcher)")
    ap.add_argument("--grid", default="4x4", help="--api render: the tile grid (Program.cpp:106-107)")
    ap.add_argument("--call-batching", type=int, default=-1, choices=[-1, 0, 1],
                    help="--api render: rmr_set_call_batching (-1 auto = on for a context that owns its stream, "
                         "the default; 0: one launch per call)")
    ap.add_argument("--launch-streams", type=int, default=-1,
                    help="rmr_set_launch_streams for every renderer context (-1: the library default; 0 off; "
                         "N >= 2: consecutive trace launches overlap on N private streams)")
    return ap.parse_args()


def scene_for_frame(cfg, frame):
    """Scene dict for a frame: static configs return the file; C5 moves the Cornell sphere
    (objects[3]) to y = 0.5 sin(2 pi f / 120)."""
    if cfg["scene"] is None:
        return None
    path = os.path.normpath(os.path.join(ROOT, "scenes", cfg["scene"]))
    if not cfg.get("animated"):
        return path
    with open(path) as f:
        sc = json.load(f)
    sc["objects"][3]["nodes"][0]["inputs"][1][1] = 0.5 * math.sin(2.0 * math.pi * frame / 120.0)
    return sc


def cpu_threads():
    """Threads for the CPU leg: every CPU this process may run on (its affinity set), capped by
    OMP_NUM_THREADS where the environment sets it. On the GPU box the harness sets 16, the host-CPU
    share of one GPU (the machine's other CPUs belong to other GPUs' jobs); in this container 8."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


def cpu_baseline(cfg, spp, seconds, threads, repeats=3):
    """CPU leg on a bounded sample of the same workload: 40 rows spread over the frame, samples 0.. of
    the same schedule. `repeats` timed runs of ~seconds/repeats each after an untimed warm-up; the
    median is reported. RM1 configs run the vectorised port (oracle/rmr_cpu_wave.c:
    the oracle's path 8 lanes at a time on AVX2, as the reference's llvmpipe JIT runs 8 invocations per
    vector; bitwise the scalar oracle, tests/test_cpu_wave.py), with the scalar oracle (the checker)
    timed beside it; RM2 / RM3 configs run the scalar oracle."""
    import statistics
    import numpy as np
    from oracle import camera, oracle
    from raymarchrenderer_amd import abi, time_schedule
    W, H = cfg["W"], cfg["H"]
    o = oracle.Oracle(oracle_tables(cfg, scene_for_frame(cfg, 0)), abi.default_params(max_bounces=cfg["bounces"]),
                      camera.default_view(W, H), W, H)
    stride = max(1, H // 40)
    rows = list(range(0, H, stride))
    # rows in bit-reversed order (any prefix is spread over the frame), each with the schedule's first
    # min(spp, 4) samples; every repeat renders the same prefix of this list again, so the repeats
    # time identical work and the median is a plain timing median
    nb = max(1, (len(rows) - 1).bit_length())
    order = sorted(range(len(rows)), key=lambda i: int(format(i, "0%db" % nb)[::-1], 2))
    ns = min(spp, 4)
    units = [(rows[i], s) for i in order for s in range(ns)]
    times = time_schedule(spp)
    wave = o.render_wave(times[0:1], rect=(0, 0, 1, 1), nthreads=1) is not None

    acc = np.zeros((H, W, 4), np.float32)   # one accumulator for every call (a fresh 33 MB array per
                                            # row call measured ~4 ms of the call's time)

    def timed(render, secs, reps, units, per_call):
        # untimed warm-up (~1/8 of the budget): the OpenMP pool and the cores' clocks settle (measured:
        # the first second of RM3 rows ran up to 10x slower than the same rows afterwards)
        t0, i = time.perf_counter(), 0
        while time.perf_counter() - t0 < secs / 8:
            y, s = units[i % len(units)]
            render(times[s:s + 1], rect=None if y is None else (0, y, W, y + 1), first_sample=s, accum=acc,
                   nthreads=threads)
            i += 1
        rates, total = [], 0
        for _ in range(reps):
            done, i = 0, 0
            t0 = time.perf_counter()
            while True:
                y, s = units[i % len(units)]
                render(times[s:s + 1], rect=None if y is None else (0, y, W, y + 1), first_sample=s, accum=acc,
                       nthreads=threads)
                done += per_call
                i += 1
                if time.perf_counter() - t0 >= secs / reps:
                    break
            rates.append(done / (time.perf_counter() - t0) / 1e6)
            total += done
        return rates, total

    scalar_impl = "scalar C restatement (oracle/rmr_oracle.c)"
    wave_impl = "AVX2 8-lane wavefront port (oracle/rmr_cpu_wave.c), bitwise the scalar oracle"
    if wave:
        # the vectorised port takes one sample of every sampled row per call (one batch shared by the
        # threads: a call per row would drain the lanes 40 times as often); the same samples. Both
        # ports are timed (half the budget each) and the faster one is the baseline: on small frames
        # (C1's 256-pixel rows) the wavefront's lane drain costs more than its vectors gain
        def render(t, rect, first_sample, accum, nthreads):
            return o.render_wave_rows(t, rows, first_sample=first_sample, accum=accum, nthreads=nthreads)
        vunits = [(None, s) for s in range(ns)]
        wr, wt = timed(render, seconds / 2, repeats, vunits, len(rows) * W)
        sr, st = timed(o.render, seconds / 2, repeats, units, W)
        if statistics.median(wr) >= statistics.median(sr):
            rates, total, impl, other = wr, wt, wave_impl, ("scalar_port", sr, st, scalar_impl)
        else:
            rates, total, impl, other = sr, st, scalar_impl, ("wave_port", wr, wt, wave_impl)
    else:
        rates, total = timed(o.render, seconds, repeats, units, W)
        impl, other = scalar_impl, None
    out = {"value": statistics.median(rates), "unit": "Msamples/s", "cores": threads, "kind": "port",
           "per_core": round(statistics.median(rates) / threads, 4), "implementation": impl,
           "repeats_msamples_per_s": [round(x, 4) for x in rates],
           "sample": "median of %d timed runs (%d samples in all) of the same work: rows y%%%d==0 of the %dx%d "
                     "frame x the schedule's first %d samples (%s), %d-thread OpenMP %s; %d threads "
                     "= every CPU of this process's affinity set, capped by OMP_NUM_THREADS (the host-CPU share of "
                     "one GPU on the GPU box)" % (repeats, total, stride, W, H, ns,
                                                  "one call per sample over all the rows" if impl == wave_impl else
                                                  "one call per row and sample, rows in bit-reversed order",
                                                  threads, impl, threads),
           "host_cpus_visible": os.cpu_count()}
    if other:
        # the other port on the same work (the scalar oracle is the checker)
        out[other[0]] = {"value": round(statistics.median(other[1]), 4),
                         "per_core": round(statistics.median(other[1]) / threads, 4),
                         "repeats_msamples_per_s": [round(x, 4) for x in other[1]], "samples": other[2],
                         "implementation": other[3]}
    ref = LLVMPIPE_PER_VCPU.get(cfg_name_of(cfg))
    if ref:
        # the reference's own path (RayMarch.glsl on Mesa llvmpipe) cannot run on the GPU box (no
        # reference sources there): its per-vCPU rate measured in the build container (BASELINE.md
        # §2, 8 vCPU), scaled to the same core count, beside the port's measured rate
        out["reference_llvmpipe_scaled"] = {
            "value": round(ref[0] * threads, 3), "per_vcpu": ref[0], "cores": threads,
            "basis": ref[1] + "; scaled linearly to %d cores, not measured on this box" % threads}
    return out


# Msamples/s per vCPU of the reference GLSL on llvmpipe (BASELINE.md §2 / SURVEY §6, 8 vCPU Xeon)
LLVMPIPE_PER_VCPU = {
    "c1": (3.65 / 8, "RM1 single sphere 256x256 1 spp: 3.5-3.8 Msamples/s on 8 vCPU"),
    "c2": (3.56 / 8, "RM1 Cornell-5 1920x1080 4 bounces: 3.56 Msamples/s on 8 vCPU"),
    "c5": (3.56 / 8, "RM1 Cornell-5 (C5's scene, static) 1920x1080 4 bounces: 3.56 Msamples/s on 8 vCPU"),
    "rm3": (5.3 / 8, "RM3 as wired 1920x1080 4 spp 16 bounces: 5.2-5.4 Msamples/s on 8 vCPU"),
    "rm2": (19.0 / 8, "RM2 simple.scene 1920x1080 4 spp 16 bounces: 18-20 Msamples/s on 8 vCPU"),
}


def cfg_name_of(cfg):
    for k, v in CONFIGS.items():
        if v is cfg:
            return k
    return None


# reference render per config (tests/golden/, llvmpipe): (file, scene it was rendered from). C4's is
# csg256's generator cut to 64 primitives (the reference's codegen does not finish 256 on llvmpipe);
# C5's is the animation's frame 0 (the sphere at y = 0 is the static Cornell-5 scene)
GOLDEN_OF = {"c1": ("img_rm1_sphere1_b1.npz", "sphere1.scene"), "c2": ("img_rm1_cornell5_b4.npz", "cornell5.scene"),
             "c3": ("img_rm1_mandelbulb_b2.npz", "mandelbulb.scene"), "c4": ("img_rm1_csg64_b4.npz", "csg64.scene"),
             "c5": ("img_rm1_cornell5_b4.npz", "cornell5.scene"), "rm3": ("img_rm3_builtin.npz", None),
             "rm2": ("img_rm2_simple.npz", "../tests/golden/scenes/simple.scene")}


def psnr_vs_reference(cfg_name, cfg, device):
    """PSNR of a converged GPU render against the reference GLSL's own converged render of the same
    scene (Mesa llvmpipe, tests/golden/, generated by oracle/glsl_ref/make_goldens.py) on the shared
    small-seed schedule. Outside the timed region."""
    import numpy as np
    from raymarchrenderer_amd import Renderer, abi, parity_schedule
    if cfg_name not in GOLDEN_OF:
        return None
    name, scene = GOLDEN_OF[cfg_name]
    g = np.load(os.path.join(ROOT, "tests", "golden", name))
    ref = g["conv"]
    H, W = ref.shape[:2]
    n = int(g["spp_conv"])
    r = Renderer(device, W, H)
    try:
        load_into(r, cfg, None if scene is None else os.path.normpath(os.path.join(ROOT, "scenes", scene)))
        r.set_params(abi.default_params(max_bounces=cfg["bounces"]))
        r.set_view(g["view"])
        r.render_spp(parity_schedule(n))
        img = r.read_accum()
    finally:
        r.close()
    a = np.clip(img[..., :3].astype(np.float64), 0, 1)
    b = np.clip(ref[..., :3].astype(np.float64), 0, 1)
    psnr = 10 * np.log10(1.0 / max(np.mean((a - b) ** 2), 1e-30))
    rel = (img[..., :3].mean() - ref[..., :3].mean()) / max(float(ref[..., :3].mean()), 1e-12)
    return {"psnr_db": round(float(psnr), 2), "mean_rel_diff": round(float(rel), 5),
            "reference": "%s on Mesa llvmpipe, %s, %dx%d, %d spp (tests/golden/%s)"
                         % ({"rm1": "RayMarch.glsl", "rm2": "RayMarch2.glsl", "rm3": "RayMarch3.glsl"}[variant_of(cfg)],
                            os.path.basename(scene) if scene else "built-in scene", W, H, n, name),
            "gpu_spp": n}


def count_pass(cfg, spp, device, n_count=8):
    """Executed SDF work of the workload, measured by the counting build of the specialised kernel
    (rmr_trace.h RMR_COUNT_FLOPS: a separate code object; same control flow and results, one atomic
    per wave and counted event, so it is timed nowhere). Runs the first n_count samples of the same
    frame (all tiles) outside the timed region; samples are identically distributed, so the per-map
    ratios hold for the whole frame. Returns per-map executed flops, transcendentals and the
    Mandelbulb-iteration share."""
    from raymarchrenderer_amd import Renderer, abi, time_schedule
    from raymarchrenderer_amd.multi_gpu import frame_tiles
    W, H = cfg["W"], cfg["H"]
    n = min(spp, n_count)
    r = Renderer(device, W, H)
    try:
        r.set_jit(1)
        r.set_instrument(abi.INSTR_COUNT_FLOPS)   # rmr_set_instrument: the counting code object
        load_into(r, cfg, scene_for_frame(cfg, 0))
        r.set_params(abi.default_params(max_bounces=cfg["bounces"]))
        r.reset_stats()
        r.render_tiles(time_schedule(n), frame_tiles(W, H, TILE), TILE)
        r.sync()
        cnt = r.counters()
        st = r.stats()
    finally:
        r.close()
    maps = float(cnt[0])
    return {"samples": "first %d of %d samples of the frame, all tiles" % (n, spp), "map_evals": int(cnt[0]),
            "flops_per_map": cnt[11] / maps, "transc_per_map": cnt[12] / maps,
            "mandelbulb_flops_per_map": cnt[13] / maps, "static_flops_per_map": st.flops_per_map,
            "launches": int(st.trace_launches)}


class _Stats:
    pass


def combined_stats(rs):
    """Kernel counters of the timed region summed over the renderer contexts (launch-averaged
    figures are then per launch of either context)."""
    sts = [r.stats() for r in rs]
    out = _Stats()
    for k in ("trace_ms", "trace_launches", "map_evals", "map_iters", "jit_launches"):
        setattr(out, k, sum(getattr(x, k) for x in sts))
    out.flops_per_map = sts[0].flops_per_map
    out.batch_maps = sum(r.counters()[14] for r in rs)   # map evals in shading batches (rmr.h counters)
    return out


def default_overlap(cfg, spp, world):
    """--overlap's default: contexts - 1 on the frame path. Four contexts where a rank's share of a
    frame is short (<= 20 M samples), two elsewhere, with 8 hardware queues:
      C1: 1,123 (two) / 1,620 (three) / 2,047 (four) / 1,403 (five) Msamples/s;
      RM2: 25,659 / 27,814 / 29,422 / 29,279; RM3: 3,094 / 3,131 / 3,132 / 3,055
      (r06za_hwq.log, r06zc_ctx45.log); the 8-rank C2 share: 6.22 / 6.15 / 6.10 ms (r06zd_predict_ctx.log);
      C2 at N = 1: 2,902 (two) against 2,889 (three) (r06zb_hwq_long.log).
    More than two contexts need GPU_MAX_HW_QUEUES above 4 (set at the top of this file): with 4, three
    were slower than two (C1 856)."""
    queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    return 3 if queues >= 8 and cfg["W"] * cfg["H"] * spp / max(1, world) <= 20e6 else 1


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """`--gpus N` without a launcher: start N rank processes of this script (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1) and return the worst exit status. The parent
    has not imported torch or touched the GPU: the ranks are fresh processes, not exec'd."""
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # a rank that fails (e.g. its rendezvous port was taken between free_port and the bind) would leave
    # the others waiting in the rendezvous: end them (the processes started here, by PID)
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc is not None and rc != 0]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(rc is not None for rc in rcs):
            return 0
        time.sleep(0.2)


class _StagedDist:
    """torch.distributed for the --share-gpu rehearsal: gloo reduces host tensors, so the frame
    reduce copies the accumulator to the host on the caller's current stream (which waits for the
    render enqueued on it), reduces there and copies the sum back. Everything else is the real
    module."""

    def __init__(self, dist):
        self._d = dist

    def __getattr__(self, k):
        return getattr(self._d, k)

    def reduce(self, t, dst=0, op=None, group=None, async_op=False):
        import torch
        host = t.cpu()   # synchronous on the current stream
        self._d.reduce(host, dst=dst, op=op if op is not None else self._d.ReduceOp.SUM, group=group)
        if self._d.get_rank(group) == dst:
            t.copy_(host.to(t.device))
        torch.cuda.current_stream().synchronize()
        return _DoneWork() if async_op else None


class _DoneWork:
    def wait(self):
        return True


def verify_last_frame(cfg, fr, times, scene, spp, device):
    """Rank 0, after the timed region: the last reduced frame against a one-context render of the
    whole frame (same scene, same seeds) — bitwise, since every rank's accumulator is zero outside
    its tiles and x + 0 = x."""
    import numpy as np
    from raymarchrenderer_amd import Renderer, abi
    from raymarchrenderer_amd.multi_gpu import frame_tiles
    W, H = cfg["W"], cfg["H"]
    got = fr.last.cpu().numpy()
    r = Renderer(device, W, H)
    try:
        load_into(r, cfg, scene)
        r.set_params(abi.default_params(max_bounces=cfg["bounces"]))
        r.render_tiles(times, frame_tiles(W, H, TILE), TILE)
        want = r.read_accum()
    finally:
        r.close()
    diff = got.view(np.uint32) != want.view(np.uint32)
    return {"bitwise_equal_to_one_context": bool(not diff.any()), "differing_words": int(diff.sum()),
            "frame_spp": spp}


DRY_W, DRY_H, DRY_TILE, DRY_SPP = 64, 48, 16, 2


def dry_run(args, cfg, rank, world):
    """CPU rehearsal of the multi-rank schedule: gloo, the CPU oracle renders each rank's tiles
    (test infrastructure standing in for librmr; nothing is measured), FrameRenderer's two-buffer
    pipeline over 3 frames, one reduce per frame. Rank 0 checks every frame against a one-process
    render of the whole frame."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from oracle import camera, oracle, scene_compile
    from raymarchrenderer_amd import abi, time_schedule
    from raymarchrenderer_amd.multi_gpu import FrameRenderer, frame_tiles
    dist_on = world > 1
    if dist_on:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    W, H, T = DRY_W, DRY_H, DRY_TILE

    def render_into(acc_np, tiles, times, sc):
        o = oracle.Oracle(oracle_tables(cfg, sc), abi.default_params(max_bounces=cfg["bounces"]), camera.default_view(W, H), W, H)
        for tx, ty in tiles:
            o.render(times, rect=(tx * T, ty * T, min(W, (tx + 1) * T), min(H, (ty + 1) * T)), accum=acc_np,
                     nthreads=2)

    cur = {}

    def render_fn(acc, tiles, times, first_sample):
        a = np.zeros((H, W, 4), np.float32)
        render_into(a, tiles, times, cur["scene"])
        acc.copy_(torch.from_numpy(a))

    accs = [torch.zeros((H, W, 4), dtype=torch.float32) for _ in range(2)]
    fr = FrameRenderer(None, accs, W, H, T, rank, world, dist if dist_on else None, render_fn=render_fn)
    ok = True
    for f in range(3):
        cur["scene"] = scene_for_frame(cfg, f)
        times = time_schedule(DRY_SPP, frame=f)
        acc = fr.frame(times)
        fr.finish()
        if rank == 0:
            want = np.zeros((H, W, 4), np.float32)
            render_into(want, frame_tiles(W, H, T), times, cur["scene"])
            ok = ok and bool(np.array_equal(acc.numpy().view(np.uint32), want.view(np.uint32)))
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_ranks": world, "backend": "gloo" if dist_on else "none",
                          "config": args.config, "frames": 3, "width": W, "height": H, "spp": DRY_SPP,
                          "tiles_per_rank": [len(frame_tiles(W, H, T)[r::world]) for r in range(world)],
                          "bitwise_equal_to_one_process": ok}), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if ok else 1


def predict_partition(args, cfg):
    """One GPU stands in for N: rank k's share of the frame (FrameRenderer's round-robin tile subset
    for rank k of N, no collective) is timed for k = 0..N-1 in turn, with two renderer contexts on two
    streams as every rank runs at N > 1. The frame at N = 1 is timed the same way. Predicted speed-up
    at N = T(1) / max_k T_k(N): the slowest rank sets the frame time (the reduce, ~0.3 ms per 1080p
    frame over xGMI, is not included). Also the sample-split alternative (every rank all tiles,
    spp / N samples): T(1) / T_split(N)."""
    import torch
    from raymarchrenderer_amd import Renderer, abi, time_schedule
    from raymarchrenderer_amd.multi_gpu import OVERLAP_GRID_RESERVE, FrameRenderer, frame_tile_costs
    W, H = cfg["W"], cfg["H"]
    spp = args.spp or cfg["spp"]
    animated = bool(cfg.get("animated"))
    n_ctx = (args.overlap if args.overlap >= 0 else 1) + 1   # renderer contexts (--overlap; default two)
    rs, streams = [], []
    for _ in range(n_ctx):
        r = Renderer(0, W, H)
        load_into(r, cfg, scene_for_frame(cfg, 0))
        r.set_params(abi.default_params(max_bounces=cfg["bounces"]))
        r.set_jit(1)
        s_ = torch.cuda.Stream()
        r.set_stream(s_.cuda_stream)
        rs.append(r)
        streams.append(s_)
    accs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(n_ctx)]
    torch.cuda.synchronize()
    cost_maps = {}   # per tile size: every tile's probe cost, probed once and sliced per rank share

    def timed(tile, rank, world, nspp):
        fr = FrameRenderer(rs, accs, W, H, tile, rank, world, None, streams=streams,
                           launch_streams=args.launch_streams if args.launch_streams >= 0 else None,
                           grid_reserve=args.grid_reserve if args.grid_reserve >= 0 else OVERLAP_GRID_RESERVE)
        if args.tile_order != "rows":
            if tile not in cost_maps:
                with torch.cuda.stream(streams[0]):
                    rs[0].bind_accum(accs[0].data_ptr(), accs[0].numel() * accs[0].element_size())
                    cost_maps[tile] = frame_tile_costs(rs[0], W, H, tile, time_schedule(2))
                    accs[0].zero_()
            # as main(): trial frames in both orders decide (cost-always: no trial), here per rank share
            fr.order_tiles_by_cost(time_schedule(2), min_spread=0.0 if args.tile_order == "cost-always" else 3.0,
                                   frame_times=None if args.tile_order == "cost-always" else time_schedule(nspp),
                                   cost_map=cost_maps[tile])
        f = [0]

        def step():
            if animated:
                load_into(fr.next_renderer(), cfg, scene_for_frame(cfg, f[0] % 120))
            fr.frame(time_schedule(nspp, frame=f[0] % 120 if animated else 0))
            f[0] += 1
        # animated: frames 0-2 first, so that both contexts have built the live-primitive kernel
        for _ in range(max(1, args.warmup) + (2 if animated else 0)):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        fr.close()
        return ms, len(fr.tiles)

    out = {"config": args.config, "width": W, "height": H, "spp": spp, "steps": args.steps, "contexts": n_ctx,
           "one_gpu_ms": {}, "tiles": {}, "sample_split": {}}
    ns = [int(x) for x in args.predict.split(",") if x.strip()]
    for tile in (32, 64):
        t1, _ = timed(tile, 0, 1, spp)
        out["one_gpu_ms"][str(tile)] = round(t1, 3)
        per_n = {}
        for n in ns:
            ms = [timed(tile, k, n, spp) for k in range(n)]
            t = [m for m, _ in ms]
            per_n[str(n)] = {"rank_ms": [round(x, 3) for x in t], "rank_tiles": [c for _, c in ms],
                             "max_over_mean": round(max(t) / (sum(t) / len(t)), 4),
                             "predicted_speedup": round(t1 / max(t), 3),
                             "predicted_efficiency": round(t1 / max(t) / n, 3)}
            print("predict tile %d N=%d: %s" % (tile, n, json.dumps(per_n[str(n)])), file=sys.stderr, flush=True)
        out["tiles"][str(tile)] = per_n
    t1 = out["one_gpu_ms"]["32"]
    for n in ns:
        if spp % n:
            continue
        ms, _ = timed(32, 0, 1, spp // n)
        out["sample_split"][str(n)] = {"rank_ms": round(ms, 3), "predicted_speedup": round(t1 / ms, 3),
                                       "note": "every rank renders every pixel with spp/N samples (not bitwise "
                                               "the one-GPU running mean: a fallback, SURVEY §8e)"}
    for r in rs:
        r.close()
    print(json.dumps({"partition_prediction": out}), flush=True)
    return 0


def api_render_bench(args, cfg):
    """--api render: the drop-in under the caller it exists for. Program.cpp:232-284 (fixed spp): for
    each tile of a 4x4 grid in spiral order, `spp` calls of Graphics::Render(time, min, max,
    currentSample), one sample each (G.cpp:314-354 -> rmr_render), no sync between calls. One step = one
    frame (Reload's zeroing, then every call). Reports Msamples/s, calls/s and where a call's time goes:
    the trace and fold kernels (HIP events around each launch) and the rest, the GPU idle between
    launches (host dispatch, copies, launch latency). Checks the frame bit for bit against one batched
    rmr_render_spp of the whole frame (same seeds): the per-call path computes the same samples."""
    import numpy as np
    import torch
    from raymarchrenderer_amd import Renderer, abi, tile_spiral, time_schedule
    W, H = cfg["W"], cfg["H"]
    spp = args.spp or cfg["spp"]
    gw, gh = (int(v) for v in args.grid.lower().split("x"))
    cw, ch = W // gw, H // gh   # Program.cpp:108-109 (a remainder is not rendered)
    order = tile_spiral(gw, gh)   # Program.cpp:113-115, 203-222
    times = time_schedule(spp)
    tl = [float(t) for t in times]
    r = Renderer(0, W, H)
    load_into(r, cfg, scene_for_frame(cfg, 0))
    r.set_params(abi.default_params(max_bounces=cfg["bounces"]))
    r.set_call_batching(args.call_batching)
    if args.launch_streams >= 0:
        r.set_launch_streams(args.launch_streams)
    rects = [((x * cw, y * ch), ((x + 1) * cw, (y + 1) * ch)) for x, y in order]

    def frame():
        r.reload()   # Program.cpp:172 (Graphics::Reload at the render's start: the accumulator zeroed)
        for mn, mx in rects:
            for s in range(spp):
                r.render(tl[s], mn, mx, s)

    for _ in range(max(1, args.warmup)):
        frame()
    r.sync()
    r.reset_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(args.steps):
        h0 = time.perf_counter()
        frame()
        host += time.perf_counter() - h0
        r.sync()
    elapsed = time.perf_counter() - t0
    st = r.stats()
    got = r.read_accum()
    calls = len(rects) * spp * args.steps
    samples = float(cw * ch * len(rects)) * spp * args.steps
    # the same frame as one batched call (checked bit for bit, then timed the same number of times)
    r.reload()
    r.render_spp(times, rect=(0, 0, cw * gw, ch * gh))
    want = r.read_accum()
    same = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
    r.sync()
    tb = time.perf_counter()
    for _ in range(args.steps):
        r.reload()
        r.render_spp(times, rect=(0, 0, cw * gw, ch * gh))
    r.sync()
    batched = samples / (time.perf_counter() - tb) / 1e6
    slots = r.launch_streams
    r.close()
    ms_step = elapsed / args.steps * 1e3
    out = {"metric": METRIC, "value": round(samples / elapsed / 1e6, 2), "unit": "Msamples/s", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
           "config": {"workload": "%s %dx%d %d spp %d bounces through rmr_render, one call per tile and sample "
                                  "(Program.cpp fixed-spp loop)" % (cfg["name"], W, H, spp, cfg["bounces"]),
                      "config": args.config, "api": "render", "grid": "%dx%d" % (gw, gh), "tile_px": [cw, ch],
                      "order": "spiral (Program.cpp:203-222)", "call_batching": args.call_batching,
                      "launch_streams": slots,
                      "width": W, "height": H, "spp": spp,
                      "max_bounces": cfg["bounces"]},
           "calls": {"per_step": len(rects) * spp, "per_s": round(calls / elapsed, 1),
                     "us_per_call": round(elapsed / calls * 1e6, 3),
                     "host_us_per_call": round(host / calls * 1e6, 3),
                     "trace_us_per_call": round(st.trace_ms / calls * 1e3, 3),
                     "fold_us_per_call": round(st.fold_ms / calls * 1e3, 3),
                     "gap_us_per_call": round((elapsed * 1e3 - st.trace_ms - st.fold_ms) / calls * 1e3, 3),
                     "jit_launches": int(st.jit_launches), "trace_launches": int(st.trace_launches),
                     "note": "gap = wall time minus the summed trace and fold kernel times (HIP events), per call: "
                             "the GPU idle between one call's kernels and the next's (with call batching a launch "
                             "serves many calls: trace_launches < calls)"},
           "batched_same_frame_msamples_per_s": round(batched, 2),
           "bitwise_equal_to_batched": same}
    print(json.dumps(out), flush=True)
    return 0 if same else 1


def api_group_bench(args, cfg):
    """--api group: the frame through librmr_group.so (include/rmr_group.h), the multi-GPU path of the C++
    host: --gpus N devices driven from this one process, the frame's 32x32 tiles dealt round-robin, two
    contexts per device, one ncclReduce per frame. Same workload, seeds and step as the headline; the
    last frame is checked bit for bit against one context's render of the whole frame."""
    import numpy as np
    from raymarchrenderer_amd import Renderer, abi, time_schedule
    from raymarchrenderer_amd.group import DeviceGroup
    W, H = cfg["W"], cfg["H"]
    spp = args.spp or cfg["spp"]
    if cfg.get("animated"):
        sys.exit("bench.py --api group: static configs only")
    scene = scene_for_frame(cfg, 0)
    prm = abi.default_params(max_bounces=cfg["bounces"])
    g = DeviceGroup(list(range(args.gpus)), W, H, tile=TILE)
    if scene is None:
        g.load_builtin(variant_of(cfg))
    else:
        g.load_scene(scene, variant_of(cfg))
    g.set_params(prm)
    g.reload()
    times = time_schedule(spp)
    for _ in range(max(1, args.warmup)):
        g.render_frame(times)
    g.sync()
    g.reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.render_frame(times)
    g.sync()
    elapsed = time.perf_counter() - t0
    per = [g.stats(m) for m in range(g.size())]
    got = g.read_frame()
    g.close()
    r = Renderer(0, W, H)
    load_into(r, cfg, scene)
    r.set_params(prm)
    r.render_spp(times)
    same = bool(np.array_equal(got.view(np.uint32), r.read_accum().view(np.uint32)))
    r.close()
    samples = float(W) * H * spp * args.steps
    out = {"metric": METRIC, "value": round(samples / elapsed / 1e6, 2), "unit": "Msamples/s", "n_gpus": args.gpus,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
           "config": {"workload": "%s %dx%d %d spp %d bounces through the single-process device group (librmr_group.so)"
                                  % (cfg["name"], W, H, spp, cfg["bounces"]), "config": args.config, "api": "group",
                      "width": W, "height": H, "spp": spp, "max_bounces": cfg["bounces"], "tile": TILE,
                      "parallelism": "tiles%d (one process, ncclCommInitAll)" % args.gpus},
           "members": [{"device": m, "trace_ms_per_step": round(s.trace_ms / args.steps, 3),
                        "trace_launches": int(s.trace_launches), "map_evals": int(s.map_evals)} for m, s in enumerate(per)],
           "bitwise_equal_to_one_context": same}
    print(json.dumps(out), flush=True)
    return 0 if same else 1


def main():
    args = parse()
    cfg = CONFIGS[args.config]
    if args.api == "group":
        if "WORLD_SIZE" in os.environ and os.environ["WORLD_SIZE"] != "1":
            sys.exit("bench.py --api group drives every GPU from one process (no launcher)")
        sys.exit(api_group_bench(args, cfg))
    if args.api == "render":
        if args.gpus != 1 or "WORLD_SIZE" in os.environ and os.environ["WORLD_SIZE"] != "1":
            sys.exit("bench.py --api render runs on one GPU (the reference's single context)")
        sys.exit(api_render_bench(args, cfg))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but the launcher started %d ranks" % (args.gpus, world))
    if args.dry_run:
        sys.exit(dry_run(args, cfg, rank, world))
    if args.predict:
        if world != 1:
            sys.exit("bench.py --predict runs on one GPU (--gpus 1)")
        sys.exit(predict_partition(args, cfg))
    W, H, BOUNCES = cfg["W"], cfg["H"], cfg["bounces"]
    spp = args.spp or cfg["spp"]
    import torch
    import torch.distributed as dist
    dist_on = world > 1
    if args.share_gpu:
        # every rank on the one GPU; RCCL refuses two ranks on one device, so the reduce runs over
        # gloo through host memory (_StagedDist). The render path is the product's.
        local_rank = 0
    torch.cuda.set_device(local_rank)
    if dist_on and args.share_gpu:
        dist.init_process_group("gloo")
        dist = _StagedDist(dist)
    elif dist_on:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    from raymarchrenderer_amd import Renderer, abi, time_schedule
    from raymarchrenderer_amd.multi_gpu import OVERLAP_GRID_RESERVE, FrameRenderer, reduce_frame
    animated = bool(cfg.get("animated"))

    # overlap: two renderer contexts on two streams; consecutive frames alternate between them, so
    # one frame's trace-kernel drain (~1.2 ms of a persistent kernel's last paths on a nearly idle
    # chip) overlaps the next frame's start (multi_gpu.FrameRenderer). Default on: a
    # renderer producing frame after frame pipelines them; it pays most where frames are short
    # (RM3 / RM2 4 spp, C1, a rank's 1/N of a frame at N > 1), where four contexts pay more again.
    overlap = args.overlap if args.overlap >= 0 else default_overlap(cfg, spp, world)
    n_ctx = overlap + 1 if overlap > 0 else 1
    rs, streams = [], []
    for _ in range(n_ctx):
        r = Renderer(local_rank, W, H)
        if n_ctx > 1 and args.launch_streams < 0:
            # overlapping contexts take no launch slots (FrameRenderer sets the same): dropped before
            # the context's torch stream exists, so the hardware queues go to the contexts' streams
            r.set_launch_streams(0)
        load_into(r, cfg, scene_for_frame(cfg, 0))
        r.set_params(abi.default_params(max_bounces=BOUNCES))
        if args.kernel:
            r.set_kernel(args.kernel)
        if args.shade_threshold:
            r.set_tuning(shade_threshold=args.shade_threshold)
        if animated:
            # the live-primitive kernel (rmr_jit.cpp) is built once the sphere first moves: build it
            # here, outside every timed step, by one tiny launch of frame 1's scene
            r.set_jit(1)
            r.load_scene(scene_for_frame(cfg, 1), "rm1")
            r.render_spp(time_schedule(1, frame=1), rect=(0, 0, 8, 8))
            r.reload()
            r.load_scene(scene_for_frame(cfg, 0), "rm1")
        elif n_ctx > 1:
            # load this context's scene kernel (hipRTC code object, module) with one tiny launch, so
            # that neither context first meets it inside the timed steps, whatever --warmup is
            r.set_jit(1)
            r.render_spp(time_schedule(1), rect=(0, 0, 8, 8))
        # every context on its own torch stream: FrameRenderer's zeroing, render and reduce are then
        # ordered on that one stream (never on a private stream the collective does not wait for)
        s_ = torch.cuda.Stream()
        r.set_stream(s_.cuda_stream)
        rs.append(r)
        streams.append(s_)
    n_acc = n_ctx if n_ctx > 1 else (2 if dist_on else 1)
    accs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(n_acc)]
    torch.cuda.synchronize()
    reserve = args.grid_reserve if args.grid_reserve >= 0 else OVERLAP_GRID_RESERVE
    fr = FrameRenderer(rs, accs, W, H, TILE, rank, world, dist if dist_on else None, streams=streams,
                       launch_streams=args.launch_streams if args.launch_streams >= 0 else None,
                       grid_reserve=reserve)
    static_times = time_schedule(spp)
    # cost order where the tiles' costs are uneven and trial frames in both orders say it is faster
    # (cost-always: without the trial; animated: the trial frames use frame 0's scene and seeds)
    tiles_reordered = (fr.order_tiles_by_cost(time_schedule(2), min_spread=0.0 if args.tile_order == "cost-always" else 3.0,
                                              frame_times=None if args.tile_order == "cost-always" else static_times)
                       if args.tile_order != "rows" else False)
    frame_no = [0]
    last = {}

    def step():
        f = frame_no[0]
        frame_no[0] += 1
        if animated:
            last["scene"], last["times"] = scene_for_frame(cfg, f % 120), time_schedule(spp, frame=f % 120)
            load_into(fr.next_renderer(), cfg, last["scene"])
        else:
            last["scene"], last["times"] = scene_for_frame(cfg, 0), static_times
        fr.frame(last["times"])

    for _ in range(args.warmup):
        step()
    fr.finish()
    torch.cuda.synchronize()
    for r in rs:
        r.reset_stats()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    fr.finish()   # every frame's reduce is inside the timed region
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = combined_stats(rs)
    per_rank = None
    reduce_ms = None
    verify = None
    if dist_on:
        if rank == 0 and not args.no_verify:
            verify = verify_last_frame(cfg, fr, last["times"], last["scene"], spp, local_rank)
        mine = torch.tensor([elapsed, st.trace_ms, float(st.trace_launches), float(st.map_evals),
                             float(len(fr.tiles))], dtype=torch.float64,
                            device="cpu" if args.share_gpu else "cuda")
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        allr = [a.cpu().tolist() for a in allr]
        elapsed = max(a[0] for a in allr)
        per_rank = [{"rank": i, "wall_ms_per_step": round(a[0] / args.steps * 1e3, 3),
                     "trace_ms_per_step": round(a[1] / args.steps, 3),
                     "trace_launches": int(a[2]), "map_evals": int(a[3]), "tiles32": int(a[4])}
                    for i, a in enumerate(allr)]
        # one frame reduce on its own (outside the timed region): what each step's collective costs
        # when nothing overlaps it
        acc = accs[0]
        with torch.cuda.stream(streams[0]):
            for _ in range(2):
                reduce_frame(acc, dist)
            torch.cuda.synchronize()
            dist.barrier()
            nrep = 5
            t1 = time.perf_counter()
            for _ in range(nrep):
                reduce_frame(acc, dist)
            torch.cuda.synchronize()
            reduce_ms = (time.perf_counter() - t1) / nrep * 1e3

    samples = float(W) * H * spp * args.steps
    value = samples / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    # overlapped frames: the per-launch event times include time the kernel waited behind the other
    # context's, so the roofline's per-launch figures come from `steps` more frames rendered one at a
    # time (each synchronised before the next starts), outside the timed region
    if n_ctx > 1:
        for r in rs:
            r.reset_stats()
        for _ in range(args.steps):
            step()
            fr.finish()
            torch.cuda.synchronize()
        st = combined_stats(rs)

    roof = None
    work_ref = None
    cp = None
    if rank == 0 and not args.no_count_pass and st.jit_launches:
        cp = count_pass(cfg, spp, local_rank)
    if st.trace_launches > 0 and st.trace_ms > 0:
        # rank 0's dominant kernel: its own map evals over its own launches. Executed flops per map
        # from the count pass (BVH / cache maps evaluate a few primitives, the Mandelbulb iterates a
        # point-dependent number of times); reference-equivalent: every primitive of the scene per
        # map, as the reference's map() evaluates them (RM1:224-231)
        per_launch_ms = st.trace_ms / st.trace_launches
        maps_per_launch = float(st.map_evals) / st.trace_launches
        if cp is not None:
            fpm = cp["flops_per_map"]
            ref_fpm = st.flops_per_map + cp["mandelbulb_flops_per_map"]
        else:
            fpm = ref_fpm = st.flops_per_map
        achieved = maps_per_launch * fpm / (per_launch_ms * 1e-3) / 1e12
        traffic = None
        tj = args.traffic_json or os.path.join(ROOT, "profiles", "traffic_%s.json" % args.config)
        if os.path.exists(tj) and world == 1 and spp == cfg["spp"]:
            try:
                with open(tj) as f:
                    traffic = json.load(f).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        roof = {"bound": "valu", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
                "peak_measured": dict(FP32_MEASURED_TFLOPS, source="tools/probes/fma_peak.hip"),
                "frac_of_measured_scalar_fma": round(achieved / FP32_MEASURED_TFLOPS["v_fma_f32"], 4),
                "kernel": ("rmr_jit_trace (hipRTC scene-specialised trace kernel)" if st.jit_launches
                           else "k_trace<RM1,persistent>"), "avg_launch_ms": round(per_launch_ms, 3),
                "map_evals_per_launch": int(st.map_evals / st.trace_launches),
                "flops_per_map": round(fpm, 2),
                "flops_basis": ("executed (count pass: %s)" % cp["samples"]) if cp else "static per-map count",
                "transcendentals_per_s": (round(maps_per_launch * cp["transc_per_map"] / (per_launch_ms * 1e-3), 1)
                                          if cp else None),
                "transcendental_peak_per_s": TRANSC_PEAK_PER_S,
                "frac_transcendental": (round(maps_per_launch * cp["transc_per_map"] / (per_launch_ms * 1e-3)
                                              / TRANSC_PEAK_PER_S, 4) if cp else None),
                "sdf_evals_per_s": round(float(st.map_evals) / (st.trace_ms * 1e-3), 1),
                # map() evaluations per map-loop lane-slot (the shading batches' certified getNormal
                # probes are map evaluations too, outside the loop: not counted here)
                "lane_utilisation": round(float(st.map_evals - st.batch_maps) / (64.0 * max(1, st.map_iters)), 4),
                "map_evals_in_shading_batches": round(float(st.batch_maps) / max(1.0, float(st.map_evals)), 4)}
        # the work a map() of the reference performs (every primitive of the scene, RM1:224-231) at the
        # same map() rate: a measure of the work skipped, not an achieved rate (it can exceed the peak)
        work_ref = {"flops_per_map": round(ref_fpm, 2),
                    "equivalent_tflops": round(maps_per_launch * ref_fpm / (per_launch_ms * 1e-3) / 1e12, 3),
                    "note": "reference-equivalent work (every primitive per map, no work skipping): not a rate "
                            "of executed flops and not compared with the peak"}
        if cfg.get("scene") and "mandelbulb" in str(cfg["scene"]):
            # the stepped map (rmr_trace.h MBStep): a map() spans several wave passes, so this is
            # map() completions per pass per lane, not the VALU lane utilisation (PMC: profiles/)
            roof["lane_utilisation_basis"] = "map() completions per wave pass / 64 (stepped Mandelbulb map)"
        if n_ctx > 1:
            roof["note"] = ("value: %d overlapping renderer contexts; avg_launch_ms and the rates: %d frames "
                            "rendered one at a time after the timed region" % (n_ctx, args.steps))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, spp, args.cpu_seconds, cpu_threads())

    parity = None
    if rank == 0 and not args.no_psnr:
        parity = psnr_vs_reference(args.config, cfg, local_rank)

    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic",
               "config": {"workload": "%s (%s semantics) %dx%d %d spp %d bounces"
                                      % (cfg["name"], {"rm1": "RayMarch.glsl", "rm2": "RayMarch2.glsl",
                                                       "rm3": "RayMarch3.glsl"}[variant_of(cfg)], W, H, spp, BOUNCES),
                          "config": args.config, "width": W, "height": H, "spp": spp, "max_bounces": BOUNCES,
                          "samples_per_step": W * H * spp, "tile": TILE, "tile_order": "cost" if tiles_reordered else "rows",
                          "tile_order_trial_ms": getattr(fr, "tile_order_trial_ms", None),
                          "parallelism": "tiles%d" % world,
                          "frame_streams": n_ctx, "grid_reserve": reserve if n_ctx > 1 else 0,
                          "launch_streams": rs[0].launch_streams},
               "roofline": roof, "cpu_baseline": cpu, "psnr_vs_reference": parity,
               "reference_equivalent_work": work_ref}
        if dist_on:
            out["multi_gpu"] = {"backend": "gloo via host (--share-gpu rehearsal)" if args.share_gpu else "nccl (RCCL)",
                                "partition": "32x32 tiles round-robin",
                                "collective": "one reduce(SUM) of the %.1f MB RGBA32F frame per step"
                                              % (W * H * 16 / 1e6),
                                "reduce_ms_standalone": round(reduce_ms, 3), "per_rank": per_rank,
                                "verify": verify}
            if args.share_gpu:
                out["n_gpus"] = 1
                out["rehearsal"] = "%d ranks sharing one GPU: a correctness rehearsal, not a measurement" % world
        print(json.dumps(out), flush=True)
    for r in rs:
        r.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
