"""The RCCL calls of the multi-GPU path, executed on a one-GPU box.

RCCL refuses two ranks on one device, so the N > 1 schedule is rehearsed on one GPU over gloo
(test_gpu_multi_rank.py) and the RCCL collective itself only runs in the driver's 8-GPU run. This
test runs RCCL here at world size 1 (backend "nccl" = RCCL on ROCm), through the product's own
pipelined schedule: a process group initialised the way bench.py initialises it (`device_id` = the
rank's GPU), then FrameRenderer with `reduce_at_world1` (its test-only switch: issue the collective
although the world has one rank) rendering three frames into two device accumulators on two renderer
contexts and streams. Each frame() zeroes its buffer, renders, and issues multi_gpu.reduce_frame's
`dist.reduce(SUM, dst=0, async_op=True)` on the frame's stream; the frame after the last context's
reuses the first buffer, so it first waits on that reduce's work handle; finish() waits for the rest. At world size 1 the reduce is
an identity, so every frame's accumulator must come back bit for bit the one-context render of the
whole frame. bench.py's `dist.all_gather` of the per-rank timing row runs too. The script runs in a
child process so its process group never meets pytest's."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import os, sys
sys.path.insert(0, os.environ["RMR_ROOT"])
import numpy as np
import torch
import torch.distributed as dist
from raymarchrenderer_amd import Renderer, abi, time_schedule
from raymarchrenderer_amd.multi_gpu import FrameRenderer, frame_tiles
from oracle import camera

W, H, TILE, SPP = 256, 192, 32, 2
scene = os.path.join(os.environ["RMR_ROOT"], "scenes", "cornell5.scene")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl"

def mk():
    r = Renderer(0, W, H)
    r.load_scene(scene, "rm1")
    r.set_params(abi.default_params(max_bounces=4))
    r.set_view(camera.default_view(W, H))
    return r

NCTX = int(os.environ["RMR_NCTX"])
NF = NCTX + 1
frames = [time_schedule(SPP, frame=f) for f in range(NF)]
rs = [mk() for _ in range(NCTX)]
accs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(NCTX)]
fr = FrameRenderer(rs, accs, W, H, TILE, 0, 1, dist, reduce_at_world1=True)
snaps = []
for f in range(NF):
    acc = fr.frame(frames[f])   # frame f + 1 renders while frame f's reduce is in flight
    i = f % NCTX
    with torch.cuda.stream(fr.streams[i]):
        fr.work[i].wait()           # stream-ordered (no host block): the copy runs after the reduce,
        snaps.append(acc.clone())   # and before frame f + NCTX zeroes the buffer on the same stream
fr.finish()
torch.cuda.synchronize()
got = [x.cpu().numpy() for x in snaps]
assert fr.reduces == NF, fr.reduces
with torch.cuda.stream(fr.streams[0]):
    row = torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64, device="cuda")
    rows = [torch.zeros_like(row)]
    dist.all_gather(rows, row)
fr.streams[0].synchronize()
assert rows[0].cpu().tolist() == [1.0, 2.0, 3.0]
for r in rs:
    r.close()

ndiff = 0
for f in range(NF):
    r1 = mk()
    r1.render_tiles(frames[f], frame_tiles(W, H, TILE), TILE)
    want = r1.read_accum()
    r1.close()
    assert np.isfinite(want).all() and (want[..., 3] == 1.0).all()
    ndiff += int((got[f].view(np.uint32) != want.view(np.uint32)).sum())
dist.destroy_process_group()
print("rccl ok: %d pipelined frames on %d contexts reduced at world 1 + all_gather, %d differing words" % (NF, NCTX, ndiff))
sys.exit(1 if ndiff else 0)
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.timeout(240)
@pytest.mark.parametrize("nctx", [2, 4])
def test_rccl_reduce_of_rendered_frame_world1(nctx):
    """Two contexts (bench.py's long frames) and four with 8 hardware queues (its short frames and the
    8-rank C2 share: bench.default_overlap) through RCCL."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RMR_ROOT=ROOT, RMR_NCTX=str(nctx))
    if nctx > 2:
        env["GPU_MAX_HW_QUEUES"] = "8"   # as bench.py sets it
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run([sys.executable, "-u", "-c", SCRIPT], capture_output=True, text=True, timeout=200,
                       env=env, cwd=ROOT)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    assert "rccl ok" in p.stdout and "0 differing words" in p.stdout, p.stdout
