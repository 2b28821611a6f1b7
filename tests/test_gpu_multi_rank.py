"""bench.py's multi-rank path on a GPU: `--gpus N --share-gpu` starts N rank processes that all render
with the HIP kernels on cuda:0 (each rank two renderer contexts on two torch streams, frames pipelined
over two accumulators, exactly the N > 1 schedule) and reduce each frame over gloo through host
memory (RCCL refuses two ranks on one device; the driver's 8-GPU run uses RCCL). Rank 0 checks the
last reduced frame bit for bit against a one-context render of the whole frame.

This is the GPU rehearsal of what the driver's scaling run does on 8 GPUs: rank spawning before any
GPU call, per-rank streams, the zero / render / reduce ordering (a renderer on a private
non-blocking stream would race the zeroing and the reduce), and the tile partition."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + list(args), capture_output=True,
                       text=True, timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("gpus,config,spp", [(2, "c2", 4), (3, "c5", 2), (8, "c2", 2)])
def test_share_gpu_ranks_reduce_bitexact(gpus, config, spp):
    out = _run("--gpus", str(gpus), "--share-gpu", "--config", config, "--spp", str(spp), "--steps", "3",
               "--warmup", "1", "--no-cpu-baseline", "--no-psnr", "--no-count-pass")
    mg = out["multi_gpu"]
    assert len(mg["per_rank"]) == gpus
    assert all(p["trace_launches"] > 0 for p in mg["per_rank"])
    assert sum(p["tiles32"] for p in mg["per_rank"]) == 60 * 34
    assert mg["verify"]["bitwise_equal_to_one_context"] is True, mg["verify"]
    assert out["config"]["frame_streams"] == 4   # a rank's share <= 20 M samples (bench.default_overlap)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_predict_partition_line():
    """bench.py --predict: per-rank shares of the N-rank tile partition timed on one GPU.
    Every rank of every N renders its own round-robin tile subset (the subsets cover the frame), and
    the predicted speed-up is consistent with the per-rank times."""
    out = _run("--config", "c2", "--spp", "2", "--predict", "2,4", "--steps", "2", "--warmup", "1")
    pp = out["partition_prediction"]
    for tile, n_tiles in (("32", 60 * 34), ("64", 30 * 17)):
        t1 = pp["one_gpu_ms"][tile]
        assert t1 > 0
        for n in ("2", "4"):
            r = pp["tiles"][tile][n]
            assert len(r["rank_ms"]) == int(n) and sum(r["rank_tiles"]) == n_tiles
            assert abs(r["predicted_speedup"] - t1 / max(r["rank_ms"])) < 0.01 * r["predicted_speedup"] + 1e-3
            assert r["max_over_mean"] >= 1.0
    assert set(pp["sample_split"]) == {"2"}   # spp 2: only N = 2 divides it


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_default_line_overlaps_frames_and_times_launches_solo():
    """bench.py's default N = 1 line: two renderer contexts whose consecutive frames overlap (the
    value), and the roofline's per-launch time from frames rendered one at a time afterwards."""
    out = _run("--config", "c1", "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-psnr")
    assert out["n_gpus"] == 1 and out["config"]["frame_streams"] == 4   # C1: four contexts (default_overlap)
    roof = out["roofline"]
    assert "one at a time" in roof["note"]
    assert 0 < roof["avg_launch_ms"] < 5 and roof["map_evals_per_launch"] > 0
    assert out["value"] > 0
