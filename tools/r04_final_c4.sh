#!/bin/bash
# Round-4 end, C4 after its shading-threshold change: GPU suite, C4 profile (r04z_c4), C4 bench line.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04z_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04z_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04z_gpu_tests.log
CONFIGS=c4 bash tools/r04_final_prof.sh || exit $?
timeout -k 10 400 python bench.py --config c4 --steps 1 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log | cut -c1-200
