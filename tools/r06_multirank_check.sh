#!/bin/bash
# the multi-rank GPU tests alone, verbose with durations (a heartbeat line per minute into the log)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
(while sleep 50; do date +%T >> gpurun_out/r06m_hb.log; done) & HB=$!
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi_rank.py -m gpu -x -v --durations=0 --timeout 300 --timeout-method thread > gpurun_out/r06m_multirank.log 2>&1; rc=$?
kill $HB
tail -25 gpurun_out/r06m_multirank.log
exit $rc
