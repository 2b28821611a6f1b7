#!/bin/bash
# round 6: the bench's default contexts by frame share (default_overlap): multi-rank GPU tests, then
# every config's default line
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi_rank.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/r06z9_multirank.log 2>&1; rc=$?
tail -8 $O/r06z9_multirank.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_benchall.sh || exit $?
for c in c1 c2 c3 c4 c5 rm2 rm3; do cp $O/bench_$c.log $O/r06z9_bench_$c.log; done
