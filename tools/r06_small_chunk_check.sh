#!/bin/bash
# round 6: GPU suite (verbose, with a heartbeat line per minute so a slow test is not taken for a hung
# run; pytest-timeout still ends a hung test) and the drop-in call-pattern probe
cd "$(dirname "$0")/.." || exit 2
TAG=${1:-r06m}
mkdir -p gpurun_out
(while sleep 50; do date +%T >> gpurun_out/${TAG}_hb.log; done) & HB=$!
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?
kill $HB
tail -22 gpurun_out/${TAG}_gpu_tests.log; [ $rc -le 1 ] || exit $rc
bash tools/api_render_probe.sh $TAG
