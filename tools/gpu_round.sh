#!/bin/bash
# GPU tests + smoke + default bench (tools/gpu_check.sh), then one C4 line and one C3 line
cd "$(dirname "$0")/.." || exit 2
bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log | cut -c1-420
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c3.log | cut -c1-420
