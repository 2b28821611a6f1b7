#!/bin/bash
# round 6 close: the GPU suite, smoke, the per-call loop with the default slots under bench.py's 8
# hardware queues, and rmr_cli under the box's 4
cd "$(dirname "$0")/.." || exit 2
TAG=${1:-r06zg}
O=gpurun_out; mkdir -p $O
(while sleep 50; do date +%T >> $O/${TAG}_hb.log; done) & HB=$!
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1; rc=$?
kill $HB
tail -3 $O/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit $?
tail -1 $O/${TAG}_smoke.log
for c in c2 rm3; do for cb in -1 0; do
  timeout -k 10 300 python bench.py --api render --config $c --steps 3 --warmup 1 --call-batching $cb > $O/${TAG}_api_${c}_cb$cb.log 2>&1 || exit $?
  echo "api render $c cb$cb: $(tail -1 $O/${TAG}_api_${c}_cb$cb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["calls"]["per_s"], d["bitwise_equal_to_batched"], d["config"]["launch_streams"])')"
done; done
CLI=raymarchrenderer_amd/rmr_cli
for m in "--per-sample" ""; do
  timeout -k 10 300 $CLI --scene scenes/cornell5.scene --size 1920x1080 --samples 64 --bounces 4 --out /tmp/cli.bmp $m > $O/${TAG}_cli_c2$m.log 2>&1 || exit $?
  echo "cli c2 [$m]: $(grep msamples $O/${TAG}_cli_c2$m.log)"
done
