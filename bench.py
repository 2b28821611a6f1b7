"""bench.py — headline benchmark: Msamples/s (pixels x spp) of the SDF ray-march path tracer.

Workload (BASELINE.json configs[1]): Cornell-5 SDF scene (scenes/cornell5.scene,
RayMarch.glsl semantics), 1920x1080, 64 spp, 4 bounces, default camera (Program.cpp:102), seed
schedule time(f, s) = 1000 f + 0.016 s. One step = one full frame at 64 spp: every pixel's 64
samples traced, folded into the RGBA32F running mean, and (N > 1) the per-rank tile accumulators
summed onto rank 0 by one RCCL reduce.

Multi-GPU: one process per GPU (torch.distributed, backend nccl = RCCL). The frame's 32x32 tiles
are dealt round-robin to the ranks; each rank renders its tiles into a zeroed full-frame
accumulator (x + 0 = x, so the reduce is exact). Total work is fixed => "scaling": "strong".

Prints ONE JSON line on rank 0 (see DESIGN.md §6 for every field).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/sec (pixels×spp) at 1920×1080; PSNR vs GLSL reference"
W, H, SPP, BOUNCES = 1920, 1080, 64, 4
TILE = 32
SCENE = os.path.join(ROOT, "scenes", "cornell5.scene")
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: peak FP32 vector (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--spp", type=int, default=SPP)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--kernel", type=int, default=0, help="0 persistent, 1 per-path")
    ap.add_argument("--shade-threshold", type=int, default=0)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_c2.json"))
    return ap.parse_args()


def cpu_baseline(seconds, spp, threads):
    """CPU oracle (oracle/liboracle.so, OpenMP) on a bounded sample of the same workload: every
    27th image row (40 rows x 1920 px) of the C2 frame, samples 0.. of the same schedule,
    repeated until ~`seconds` of CPU time."""
    from oracle import camera, oracle, scene_compile
    from raymarchrenderer_amd import abi, time_schedule
    t = scene_compile.load_scene_file(SCENE, "rm1")
    o = oracle.Oracle(t, abi.default_params(max_bounces=BOUNCES), camera.default_view(W, H), W, H)
    rows = list(range(0, H, 27))
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
            "sample": "%d samples: rows y%%27==0 of the C2 1920x1080 frame, 1 spp per row pass, "
                      "%d-thread OpenMP C restatement (oracle/rmr_oracle.c)" % (done, threads)}


def main():
    args = parse()
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

    r = Renderer(local_rank, W, H)
    r.load_scene(SCENE, "rm1")
    r.set_params(abi.default_params(max_bounces=BOUNCES))
    if args.kernel:
        r.set_kernel(args.kernel)
    if args.shade_threshold:
        r.set_tuning(shade_threshold=args.shade_threshold)
    from raymarchrenderer_amd.multi_gpu import FrameRenderer
    stream = torch.cuda.current_stream()
    r.set_stream(stream.cuda_stream)
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    fr = FrameRenderer(r, acc, W, H, TILE, rank, world, dist if dist_on else None)
    times = time_schedule(args.spp)

    def step():
        fr.frame(times)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    r.reset_stats()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = r.stats()
    if dist_on:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        # dominant-kernel numbers of rank 0 are reported; map evals summed for the roofline
        me = torch.tensor([st.map_evals, st.trace_launches], dtype=torch.float64, device="cuda")
        dist.all_reduce(me, op=dist.ReduceOp.SUM)
        total_maps = float(me[0].item())
    else:
        total_maps = float(st.map_evals)

    samples = float(W) * H * args.spp * args.steps
    value = samples / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    roof = None
    if st.trace_launches > 0 and st.trace_ms > 0:
        per_launch_ms = st.trace_ms / st.trace_launches
        flops_per_launch = float(st.map_evals) / st.trace_launches * st.flops_per_map
        achieved = flops_per_launch / (per_launch_ms * 1e-3) / 1e12
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                with open(args.traffic_json) as f:
                    traffic = json.load(f).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        roof = {"bound": "valu", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
                "kernel": "k_trace<RM1,persistent>", "avg_launch_ms": round(per_launch_ms, 3),
                "map_evals_per_launch": int(st.map_evals / st.trace_launches),
                "flops_per_map": st.flops_per_map,
                "sdf_evals_per_s": round(float(st.map_evals) / (st.trace_ms * 1e-3), 1)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        cpu = cpu_baseline(args.cpu_seconds, args.spp, threads)

    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic",
               "config": {"workload": "C2 Cornell-5 SDF (RayMarch.glsl semantics) 1920x1080 %d spp %d bounces"
                                      % (args.spp, BOUNCES),
                          "width": W, "height": H, "spp": args.spp, "max_bounces": BOUNCES,
                          "samples_per_step": W * H * args.spp, "tile": TILE,
                          "parallelism": "tiles%d" % world},
               "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    r.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
