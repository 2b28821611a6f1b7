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

Multi-GPU: one process per GPU (torch.distributed, backend nccl = RCCL). The frame's 32x32 tiles
are dealt round-robin to the ranks; each rank renders its tiles into a zeroed full-frame
accumulator (x + 0 = x, so the reduce is exact); frame f's reduce overlaps frame f + 1's render
(two accumulators). Total work is fixed => "scaling": "strong".

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

METRIC = "Msamples/sec (pixels×spp) at 1920×1080; PSNR vs GLSL reference"
TILE = 32
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: peak FP32 vector (spec)

CONFIGS = {
    "c1": dict(scene="sphere1.scene", W=256, H=256, spp=1, bounces=1, name="C1 single-sphere SDF"),
    "c2": dict(scene="cornell5.scene", W=1920, H=1080, spp=64, bounces=4, name="C2 Cornell-5 SDF"),
    "c3": dict(scene="mandelbulb.scene", W=1920, H=1080, spp=128, bounces=2, name="C3 Mandelbulb SDF"),
    "c4": dict(scene="csg256.scene", W=3840, H=2160, spp=256, bounces=4, name="C4 256-prim CSG union"),
    "c5": dict(scene="cornell5.scene", W=1920, H=1080, spp=512, bounces=4, name="C5 animated Cornell-5",
               animated=True),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override the config's spp")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-psnr", action="store_true", help="skip the converged PSNR check vs the reference render")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--kernel", type=int, default=0, help="0 persistent, 1 per-path")
    ap.add_argument("--shade-threshold", type=int, default=0)
    ap.add_argument("--traffic-json", default="")
    ap.add_argument("--overlap", action="store_true",
                    help="two renderer contexts on two streams: consecutive frames overlap on the GPU "
                         "(measured +0.9%% at N=1; the per-launch event times then include waiting)")
    return ap.parse_args()


def scene_for_frame(cfg, frame):
    """Scene dict for a frame: static configs return the file; C5 moves the Cornell sphere
    (objects[3]) to y = 0.5 sin(2 pi f / 120)."""
    path = os.path.join(ROOT, "scenes", cfg["scene"])
    if not cfg.get("animated"):
        return path
    with open(path) as f:
        sc = json.load(f)
    sc["objects"][3]["nodes"][0]["inputs"][1][1] = 0.5 * math.sin(2.0 * math.pi * frame / 120.0)
    return sc


def cpu_baseline(cfg, spp, seconds, threads):
    """CPU oracle (oracle/liboracle.so, OpenMP) on a bounded sample of the same workload: 40 rows
    spread over the frame, samples 0.. of the same schedule, repeated until ~`seconds` pass."""
    from oracle import camera, oracle, scene_compile
    from raymarchrenderer_amd import abi, time_schedule
    W, H = cfg["W"], cfg["H"]
    sc = scene_for_frame(cfg, 0)
    t = scene_compile.load_scene_file(sc, "rm1") if isinstance(sc, str) else scene_compile.compile_scene(sc, "rm1")
    o = oracle.Oracle(t, abi.default_params(max_bounces=cfg["bounces"]), camera.default_view(W, H), W, H)
    stride = max(1, H // 40)
    rows = list(range(0, H, stride))
    times = time_schedule(spp)
    done = 0
    t0 = time.perf_counter()
    k = 0
    while True:
        y = rows[k % len(rows)]
        s = (k // len(rows)) % spp
        o.render(times[s:s + 1], rect=(0, y, W, y + 1), first_sample=s, nthreads=threads)
        done += W
        k += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": "%d samples: rows y%%%d==0 of the %dx%d frame, 1 spp per row pass, %d-thread OpenMP C "
                      "restatement (oracle/rmr_oracle.c)" % (done, stride, W, H, threads)}


GOLDEN_OF = {"c1": "img_rm1_sphere1_b1.npz", "c2": "img_rm1_cornell5_b4.npz"}


def psnr_vs_reference(cfg_name, cfg, device):
    """PSNR of a converged GPU render against the reference GLSL's own converged render of the same
    scene (Mesa llvmpipe, tests/golden/, generated by oracle/glsl_ref/make_goldens.py) on the shared
    small-seed schedule. Outside the timed region; None for configs without one."""
    import numpy as np
    from raymarchrenderer_amd import Renderer, abi, parity_schedule
    name = GOLDEN_OF.get(cfg_name)
    if not name:
        return None
    g = np.load(os.path.join(ROOT, "tests", "golden", name))
    ref = g["conv"]
    H, W = ref.shape[:2]
    n = int(g["spp_conv"])
    r = Renderer(device, W, H)
    try:
        r.load_scene(os.path.join(ROOT, "scenes", cfg["scene"]), "rm1")
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
            "reference": "RayMarch.glsl on Mesa llvmpipe, %dx%d, %d spp (tests/golden/%s)" % (W, H, n, name),
            "gpu_spp": n}


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
    return out


def main():
    args = parse()
    cfg = CONFIGS[args.config]
    W, H, BOUNCES = cfg["W"], cfg["H"], cfg["bounces"]
    spp = args.spp or cfg["spp"]
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    dist_on = world > 1
    if dist_on:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    from raymarchrenderer_amd import Renderer, abi, time_schedule

    # --overlap: two renderer contexts on two streams; consecutive frames alternate between them,
    # so one frame's trace-kernel drain overlaps the next frame's start (multi_gpu.FrameRenderer)
    n_ctx = 2 if (args.overlap and not cfg.get("animated")) else 1
    rs, streams = [], []
    for _ in range(n_ctx):
        r = Renderer(local_rank, W, H)
        r.load_scene(scene_for_frame(cfg, 0), "rm1")
        r.set_params(abi.default_params(max_bounces=BOUNCES))
        if args.kernel:
            r.set_kernel(args.kernel)
        if args.shade_threshold:
            r.set_tuning(shade_threshold=args.shade_threshold)
        s_ = torch.cuda.Stream() if n_ctx > 1 else torch.cuda.current_stream()
        r.set_stream(s_.cuda_stream)
        rs.append(r)
        streams.append(s_)
    from raymarchrenderer_amd.multi_gpu import FrameRenderer
    n_acc = 2 if (dist_on or n_ctx > 1) else 1
    accs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(n_acc)]
    torch.cuda.synchronize()
    fr = FrameRenderer(rs, accs, W, H, TILE, rank, world, dist if dist_on else None,
                       streams=streams if n_ctx > 1 else None)
    animated = bool(cfg.get("animated"))
    static_times = time_schedule(spp)
    frame_no = [0]

    def step():
        f = frame_no[0]
        frame_no[0] += 1
        if animated:
            fr.next_renderer().load_scene(scene_for_frame(cfg, f % 120), "rm1")
            fr.frame(time_schedule(spp, frame=f % 120))
        else:
            fr.frame(static_times)

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
    if dist_on:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    samples = float(W) * H * spp * args.steps
    value = samples / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    roof = None
    if st.trace_launches > 0 and st.trace_ms > 0:
        # rank 0's dominant kernel: its own map evals over its own launches
        per_launch_ms = st.trace_ms / st.trace_launches
        flops_per_launch = float(st.map_evals) / st.trace_launches * st.flops_per_map
        achieved = flops_per_launch / (per_launch_ms * 1e-3) / 1e12
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
                "kernel": ("rmr_jit_trace (hipRTC scene-specialised trace kernel)" if st.jit_launches
                           else "k_trace<RM1,persistent>"), "avg_launch_ms": round(per_launch_ms, 3),
                "map_evals_per_launch": int(st.map_evals / st.trace_launches),
                "flops_per_map": st.flops_per_map,
                "sdf_evals_per_s": round(float(st.map_evals) / (st.trace_ms * 1e-3), 1),
                "lane_utilisation": round(float(st.map_evals) / (64.0 * max(1, st.map_iters)), 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        cpu = cpu_baseline(cfg, spp, args.cpu_seconds, threads)

    parity = None
    if rank == 0 and not args.no_psnr:
        parity = psnr_vs_reference(args.config, cfg, local_rank)

    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic",
               "config": {"workload": "%s (RayMarch.glsl semantics) %dx%d %d spp %d bounces"
                                      % (cfg["name"], W, H, spp, BOUNCES),
                          "config": args.config, "width": W, "height": H, "spp": spp, "max_bounces": BOUNCES,
                          "samples_per_step": W * H * spp, "tile": TILE, "parallelism": "tiles%d" % world,
                          "frame_streams": n_ctx},
               "roofline": roof, "cpu_baseline": cpu, "psnr_vs_reference": parity}
        print(json.dumps(out), flush=True)
    for r in rs:
        r.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
