#!/bin/bash
# Round-4 end: bench lines of C2 / C5 / RM3 / C4 again, now that their traffic_<cfg>.json come from the
# same-HEAD profiles (bench.py reads them at run time).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | cut -c1-120
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 2 > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5.log | cut -c1-120
timeout -k 10 300 python bench.py --config rm3 --steps 30 --warmup 2 > gpurun_out/bench_rm3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_rm3.log | cut -c1-120
timeout -k 10 400 python bench.py --config c4 --steps 1 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log | cut -c1-120
