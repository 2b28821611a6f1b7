#!/bin/bash
# every BASELINE config once (1 GPU) plus the reference's own kernels, each with its CPU leg (the oracle
# on the host cores, a bounded sample of the same frame); logs in gpurun_out/bench_<cfg>.log
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | cut -c1-330
# short frames (C1 0.1 ms, RM2 1 ms, RM3 3 ms) get enough steps for the two overlapping contexts'
# steady state (3 steps are mostly pipeline fill)
for c in c1 c3 c5 rm3 rm2; do
  st=3; [ $c = c1 ] && st=200; [ $c = rm3 ] && st=30; [ $c = rm2 ] && st=60; [ $c = c3 ] && st=5
  timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 > gpurun_out/bench_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$c.log | cut -c1-330
done
timeout -k 10 400 python bench.py --config c4 --steps 1 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log | cut -c1-330
