#!/bin/bash
# Round-4 end, after the 7-wave setting of the approximate RM1 and RM3 kernels: GPU suite, then the
# profiles (r04z_<cfg>) and bench lines of the configs it touches (C2, C5, RM3).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04z_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04z_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04z_gpu_tests.log
CONFIGS="c2 c5 rm3" bash tools/r04_final_prof.sh || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | cut -c1-200
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 2 > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5.log | cut -c1-200
timeout -k 10 300 python bench.py --config rm3 --steps 30 --warmup 2 > gpurun_out/bench_rm3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_rm3.log | cut -c1-200
