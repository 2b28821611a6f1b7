"""The RCCL calls of the multi-GPU path, executed on a one-GPU box.

RCCL refuses two ranks on one device, so the N > 1 schedule is rehearsed on one GPU over gloo
(test_gpu_multi_rank.py) and the RCCL collective itself only runs in the driver's 8-GPU run. This
test runs RCCL here at world size 1 (backend "nccl" = RCCL on ROCm): a process group initialised the
way bench.py initialises it (`device_id` = the rank's GPU), a frame rendered by FrameRenderer on its
torch stream into a device accumulator, then the two collectives bench.py's N > 1 path issues on
device tensors — `dist.reduce(SUM, dst=0)` of the accumulator (multi_gpu.reduce_frame, ordered on the
frame's stream, async work handle waited) and `dist.all_gather` of the per-rank timing row. At world
size 1 the reduce is an identity, so the accumulator must come back bit for bit the one-context render
of the whole frame. The script runs in a child process so its process group never meets pytest's."""
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

times = time_schedule(SPP)
r = mk()
accs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
fr = FrameRenderer([r], accs, W, H, TILE, 0, 1, dist)
fr.frame(times)
acc = fr.finish()
s = fr.streams[0]
with torch.cuda.stream(s):
    work = dist.reduce(acc, dst=0, op=dist.ReduceOp.SUM, async_op=True)
    work.wait()
    row = torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64, device="cuda")
    rows = [torch.zeros_like(row)]
    dist.all_gather(rows, row)
s.synchronize()
got = acc.cpu().numpy()
assert rows[0].cpu().tolist() == [1.0, 2.0, 3.0]
r.close()

r1 = mk()
r1.render_tiles(times, frame_tiles(W, H, TILE), TILE)
want = r1.read_accum()
r1.close()
dist.destroy_process_group()
diff = got.view(np.uint32) != want.view(np.uint32)
assert np.isfinite(want).all() and (want[..., 3] == 1.0).all()
print("rccl ok: reduce + all_gather at world 1, %d differing words" % int(diff.sum()))
sys.exit(1 if diff.any() else 0)
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_rccl_reduce_of_rendered_frame_world1():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RMR_ROOT=ROOT)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run([sys.executable, "-u", "-c", SCRIPT], capture_output=True, text=True, timeout=200,
                       env=env, cwd=ROOT)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    assert "rccl ok" in p.stdout and "0 differing words" in p.stdout, p.stdout
