#!/bin/bash
# round 6: launch slots on by default (2): the GPU suite, then bench lines (two contexts, the default;
# one context), the drop-in call pattern with and without call batching, and the C++ host's loops
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06q_launch_streams_default.log
mkdir -p $O
(while sleep 50; do date +%T >> $O/r06q_hb.log; done) & HB=$!
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/r06q_gpu_tests.log 2>&1; rc=$?
kill $HB
tail -3 $O/r06q_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
F="--no-cpu-baseline --no-psnr --no-count-pass"
for c in c1 rm3 rm2 c2 c3; do
  st=3; [ $c = c1 ] && st=200; [ $c = rm3 ] && st=30; [ $c = rm2 ] && st=60
  for v in "" "--overlap 0"; do
    timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 $F $v > $O/r06q_tmp.log 2>&1 || exit $?
    echo "$c [$v]: $(tail -1 $O/r06q_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["launch_streams"])')" | tee -a $L
  done
done
for c in c2 rm3; do for cb in -1 0; do
  timeout -k 10 300 python bench.py --api render --config $c --steps 3 --warmup 1 --call-batching $cb > $O/r06q_api_${c}_cb$cb.log 2>&1 || exit $?
  echo "api render $c cb$cb: $(tail -1 $O/r06q_api_${c}_cb$cb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["calls"]["per_s"], d["bitwise_equal_to_batched"], d["config"]["launch_streams"])')" | tee -a $L
done; done
CLI=raymarchrenderer_amd/rmr_cli
for m in "--per-sample" ""; do
  timeout -k 10 300 $CLI --scene scenes/cornell5.scene --size 1920x1080 --samples 64 --bounces 4 --out /tmp/cli.bmp $m > $O/r06q_cli_c2$m.log 2>&1 || exit $?
  echo "cli c2 [$m]: $(grep msamples $O/r06q_cli_c2$m.log)" | tee -a $L
done
