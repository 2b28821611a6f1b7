"""bench.py's multi-rank launch on the CPU: `--gpus N` without a launcher starts N rank processes
(RANK / WORLD_SIZE / MASTER_* on 127.0.0.1) and `--dry-run` runs the frame schedule over gloo with the
CPU oracle as each rank's renderer. Rank 0's frames must equal a one-process render bit for bit
(the tile partition + one reduce per frame is exact). Nothing here touches a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args), capture_output=True,
                       text=True, timeout=600, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout      # one JSON line, from rank 0 only
    return json.loads(lines[0])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("gpus,config", [(2, "c2"), (3, "c5"), (8, "c2")])
def test_bench_spawns_ranks_and_reduces_exactly(gpus, config):
    """World 8 rehearses the driver's N = 8 scaling run (8 gloo ranks on the CPU, 12 tiles: uneven shares)."""
    out = _run("--gpus", str(gpus), "--dry-run", "--config", config)
    assert out["dry_run"] is True
    assert out["n_ranks"] == gpus and out["backend"] == "gloo"
    assert out["bitwise_equal_to_one_process"] is True
    assert sum(out["tiles_per_rank"]) == (64 // 16) * (48 // 16)


def test_bench_rejects_mismatched_launcher():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode != 0 and "--gpus 2" in p.stderr


def test_default_contexts_and_hardware_queues(monkeypatch):
    """bench.default_overlap: four overlapping contexts for a rank's frame share of <= 20 M samples
    when the process has 8 hardware queues (bench.py raises GPU_MAX_HW_QUEUES to 8 at import), two
    otherwise; with HIP's default 4 queues always two (three were slower: DESIGN.md §5)."""
    sys.path.insert(0, ROOT)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    import importlib
    import bench
    bench = importlib.reload(bench)   # (the module-level raise runs again with this environment)
    assert int(os.environ["GPU_MAX_HW_QUEUES"]) == 8
    c = bench.CONFIGS
    assert bench.default_overlap(c["c1"], 1, 1) == 3
    assert bench.default_overlap(c["rm2"], 4, 1) == 3 and bench.default_overlap(c["rm3"], 4, 1) == 3
    assert bench.default_overlap(c["c2"], 64, 1) == 1 and bench.default_overlap(c["c2"], 64, 4) == 1
    assert bench.default_overlap(c["c2"], 64, 8) == 3   # the 8-rank share: 16.6 M samples
    assert bench.default_overlap(c["c4"], 256, 8) == 1
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    assert bench.default_overlap(c["c1"], 1, 1) == 1
