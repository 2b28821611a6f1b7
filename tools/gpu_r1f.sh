#!/bin/bash
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_jit.log 2>&1 || exit $?
tail -1 gpurun_out/bench_jit.log | cut -c1-260
RMR_JIT=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_aot.log 2>&1 || exit $?
tail -1 gpurun_out/bench_aot.log | cut -c1-260
timeout -k 10 300 python tools/tune.py --spp 16 --configs '[{"T":10,"TR":0},{"T":16,"TR":4},{"T":16,"TR":8},{"T":20,"TR":4},{"T":24,"TR":4},{"T":12,"TR":4},{"T":10,"TR":0},{"T":16,"TR":4}]' > gpurun_out/tune_jit.log 2>&1 || exit $?
cat gpurun_out/tune_jit.log | cut -c1-200
