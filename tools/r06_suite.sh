#!/bin/bash
# the GPU suite (verbose, heartbeat), smoke, and the default bench line
cd "$(dirname "$0")/.." || exit 2
TAG=${1:-r06w}
O=gpurun_out; mkdir -p $O
(while sleep 50; do date +%T >> $O/${TAG}_hb.log; done) & HB=$!
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1; rc=$?
kill $HB
tail -3 $O/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit $?
tail -1 $O/${TAG}_smoke.log
timeout -k 10 300 python bench.py > $O/${TAG}_bench_c2.log 2>&1 || exit $?
tail -1 $O/${TAG}_bench_c2.log | cut -c1-300
