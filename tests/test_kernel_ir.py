"""The generated trace kernels carry no undefined values into their loops (CPU; hipcc cross-compiles).

Round 4's forced-wave glass_test miscompute came from `Lane L;` in trace_main: most lane fields were
never written before the persistent loop, so the optimised IR had `phi [undef, %entry]` at the loop
header for each of them, and the register allocator's live-range splitting could legally drop a
lane's value on the paths that came from the entry. trace_main now defines every field (opaque inline
asm values, rmr_trace.h lane_define: no constant for the optimiser to propagate, so no extra register
pressure) and the cache kernels' full-map outputs. This test compiles one kernel of every class the
hipRTC specialiser generates to LLVM IR with the hipRTC options and checks that no PHI node takes an
undef or poison input, and that the occupancy targets still hold without scratch spills where the
kernel had none."""
import os
import re
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

from raymarchrenderer_amd.renderer import jit_compile_scene

from .conftest import GOLDEN, ROOT, SCENES

HIPCC = "/opt/rocm/bin/hipcc"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
# rmr_jit.cpp kOptions
OPTS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-Wno-unused-function",
        "-fno-slp-vectorize", "-DRMR_MANDELBULB_INLINE=1"]
CASES = [   # name, scene, variant, extra -D options, spill-free
    ("cornell5_cert", os.path.join(SCENES, "cornell5.scene"), "rm1", [], True),
    ("mandelbulb_stepped", os.path.join(SCENES, "mandelbulb.scene"), "rm1", [], True),
    ("csg256_cache", os.path.join(SCENES, "csg256.scene"), "rm1", [], True),
    ("rm2_simple", os.path.join(GOLDEN, "scenes", "simple.scene"), "rm2", [], True),
    ("rm3_builtin", None, "rm3", [], True),
    ("glass_prog", os.path.join(GOLDEN, "scenes", "glass_test.scene"), "rm1", [], False),
    ("glass_prog_6waves", os.path.join(GOLDEN, "scenes", "glass_test.scene"), "rm1", ["-DRMR_PROG_WAVES=6"], False),
]


def _source(tmp, scene, variant, monkeypatch):
    d = tmp / "dump"
    d.mkdir(exist_ok=True)
    monkeypatch.setenv("RMR_JIT_DUMP", str(d))
    monkeypatch.setenv("RMR_JIT_CACHE", str(tmp / "cache"))
    key = jit_compile_scene(scene, variant, diag=True)
    return (d / (key + ".hip")).read_text()


def _compile(src_path, extra, what):
    src = open(src_path).read()
    opts = list(OPTS)
    for line in src.splitlines():
        if line.startswith("//@opts "):
            opts += line[8:].split()
    inc = ["-I", os.path.join(ROOT, "raymarchrenderer_amd", "csrc"), "-I", os.path.join(ROOT, "include")]
    base = [HIPCC] + opts + extra + inc + ["--offload-device-only", "-x", "hip", src_path]
    if what == "ir":
        out = src_path + ".ll"
        subprocess.run(base[:-3] + ["-S", "-emit-llvm", "-o", out] + base[-3:], check=True, capture_output=True)
        return open(out).read()
    out = src_path + ".o"
    subprocess.run(base[:-3] + ["--no-gpu-bundle-output", "-c", "-o", out] + base[-3:], check=True, capture_output=True)
    notes = subprocess.run([READELF, "--notes", out], check=True, capture_output=True, text=True).stdout
    return {k: int(v) for k, v in re.findall(r"\.(vgpr_spill_count|private_segment_fixed_size):\s+(\d+)", notes)}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_generated_kernels_have_no_undef_phis(tmp_path, monkeypatch):
    jobs = []
    for name, scene, variant, extra, spill_free in CASES:
        p = tmp_path / (name + ".hip")
        p.write_text(_source(tmp_path, scene, variant, monkeypatch))
        jobs.append((name, str(p), extra, spill_free))
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 2)) as ex:
        irs = list(ex.map(lambda j: _compile(j[1], j[2], "ir"), jobs))
        notes = list(ex.map(lambda j: _compile(j[1], j[2], "obj"), jobs))
    for (name, _, _, spill_free), ir, nt in zip(jobs, irs, notes):
        bad = [ln.strip() for ln in ir.splitlines() if " phi " in ln and re.search(r"\b(undef|poison)\b", ln)]
        assert not bad, "%s: %d PHIs with undef/poison inputs, e.g. %s" % (name, len(bad), bad[:3])
        if spill_free:
            assert nt.get("vgpr_spill_count", 0) == 0, (name, nt)
