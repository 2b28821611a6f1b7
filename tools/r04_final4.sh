#!/bin/bash
# Round-4 end, after the Cornell-5 shading threshold: GPU suite, C2 / C5 profiles and bench lines.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04z_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04z_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04z_gpu_tests.log
CONFIGS="c2 c5" bash tools/r04_final_prof.sh || exit $?
python tools/summarize_profile.py r04z_c2 c2 > /dev/null && python tools/summarize_profile.py r04z_c5 c5 > /dev/null || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | cut -c1-120
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 2 > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5.log | cut -c1-120
