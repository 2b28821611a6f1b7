"""Multi-rank path on CPU (gloo, world size 2): the tile partition + one reduce reproduce the
single-process frame bit for bit. The per-rank renderer here is the CPU oracle (test
infrastructure); on the GPU box bench.py runs the same partition through librmr over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import camera, oracle, scene_compile
from raymarchrenderer_amd import abi, time_schedule
from raymarchrenderer_amd.multi_gpu import FrameRenderer, frame_tiles, reduce_frame, tile_partition

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, TILE = 40, 24, 16


def _render_tiles(tiles, times):
    t = scene_compile.load_scene_file(os.path.join(ROOT, "scenes", "cornell5.scene"), "rm1")
    o = oracle.Oracle(t, abi.default_params(max_bounces=3), camera.default_view(W, H), W, H)
    acc = np.zeros((H, W, 4), np.float32)
    for tx, ty in tiles:
        o.render(times, rect=(tx * TILE, ty * TILE, min(W, (tx + 1) * TILE), min(H, (ty + 1) * TILE)),
                 accum=acc, nthreads=2)
    return acc


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    times = time_schedule(2)
    acc = torch.from_numpy(_render_tiles(tile_partition(W, H, TILE, rank, world), times))
    reduce_frame(acc, dist)
    if rank == 0:
        q.put(acc.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_partition_covers_frame_once():
    for world in (1, 2, 3, 8):
        parts = [set(map(tuple, tile_partition(1920, 1080, 32, r, world))) for r in range(world)]
        assert sum(len(p) for p in parts) == len(frame_tiles(1920, 1080, 32))
        assert set().union(*parts) == set(frame_tiles(1920, 1080, 32))
        sizes = [len(p) for p in parts]
        assert max(sizes) - min(sizes) <= 1


@pytest.mark.timeout(300)
def test_gloo_two_ranks_reduce_is_exact():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _render_tiles(frame_tiles(W, H, TILE), time_schedule(2))
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def _oracle_into(acc, tiles, times, first_sample):
    acc.copy_(torch.from_numpy(_render_tiles(tiles, times)))


def _pipelined_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    accs = [torch.zeros((H, W, 4), dtype=torch.float32) for _ in range(2)]
    fr = FrameRenderer(None, accs, W, H, TILE, rank, world, dist, render_fn=_oracle_into)
    for f in range(3):   # frame 2 reuses buffer 0 after waiting for frame 0's reduce
        fr.frame(time_schedule(2, frame=f))
    last = fr.finish()
    if rank == 0:
        q.put((last.numpy().copy(), accs[1].numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_two_ranks_pipelined_frames_exact():
    """FrameRenderer's two-buffer schedule (async reduce of frame f while frame f + 1 renders):
    every frame's reduced image equals the single-process render."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    f2, f1 = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for got, f in ((f2, 2), (f1, 1)):
        want = _render_tiles(frame_tiles(W, H, TILE), time_schedule(2, frame=f))
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f


@pytest.mark.gpu
def test_overlapped_frames_two_streams_bitexact():
    """bench.py --overlap: frames alternate between two renderer contexts on two HIP streams
    (FrameRenderer(renderer=[r0, r1], streams=[s0, s1])), so consecutive frames run concurrently.
    Every frame's image equals the one-context, one-stream schedule bit for bit."""
    from raymarchrenderer_amd import Renderer
    W, H, tile = 96, 64, 32
    scene = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scenes", "cornell5.scene")

    def run(n_ctx):
        rs, streams = [], []
        for _ in range(n_ctx):
            r = Renderer(0, W, H)
            r.set_jit(1)
            r.load_scene(scene, "rm1")
            r.set_params(abi.default_params(max_bounces=4))
            s = torch.cuda.Stream() if n_ctx > 1 else torch.cuda.current_stream()
            r.set_stream(s.cuda_stream)
            rs.append(r)
            streams.append(s)
        accs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
        ls0 = rs[0].launch_streams   # the library's default launch slots (2, or 4 with 8 hardware queues)
        assert ls0 >= 2 and all(r.launch_streams == ls0 for r in rs)
        fr = FrameRenderer(rs, accs, W, H, tile, 0, 1, streams=streams if n_ctx > 1 else None)
        # two overlapping contexts take no launch slots (rmr.h rmr_set_launch_streams); one keeps them
        assert all(r.launch_streams == (0 if n_ctx > 1 else ls0) for r in rs)
        out = []
        for f in range(4):
            acc = fr.frame(time_schedule(3, frame=f))
            if f % 2 == 1:   # both buffers hold finished frames after the odd ones
                fr.finish()
                torch.cuda.synchronize()
                out.append(accs[0].cpu().numpy().view(np.uint32).copy())
                out.append(acc.cpu().numpy().view(np.uint32).copy())
        fr.close()
        assert all(r.launch_streams == ls0 for r in rs)   # given back at close()
        for r in rs:
            r.close()
        return out

    one, two = run(1), run(2)
    for a, b in zip(one, two):
        assert np.array_equal(a, b)
