#!/bin/bash
# every BASELINE config once (1 GPU) plus the reference's own kernels; logs in gpurun_out/bench_<cfg>.log
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | cut -c1-330
for c in c1 c3 c5 rm3 rm2; do
  timeout -k 10 300 python bench.py --config $c --warmup 2 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$c.log | cut -c1-330
done
timeout -k 10 400 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log | cut -c1-330
