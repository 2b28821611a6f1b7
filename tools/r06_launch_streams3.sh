#!/bin/bash
# round 6: launch slots with a 64-workgroup reserve for the folds: the drop-in call pattern and the C++
# host's loops with slots (default) and without (--launch-streams 0), one context per bench line
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06r_launch_streams_reserve.log
mkdir -p $O
for c in rm3 c2; do for cb in -1 0; do for ls in 0 2; do
  timeout -k 10 300 python bench.py --api render --config $c --steps 3 --warmup 1 --call-batching $cb --launch-streams $ls > $O/r06r_tmp.log 2>&1 || exit $?
  echo "api render $c cb$cb ls$ls: $(tail -1 $O/r06r_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["calls"]["per_s"], d["calls"]["trace_launches"], d["bitwise_equal_to_batched"])')" | tee -a $L
done; done; done
F="--no-cpu-baseline --no-psnr --no-count-pass"
for c in c1 rm3 rm2; do
  st=30; [ $c = c1 ] && st=200; [ $c = rm2 ] && st=60
  for v in "--overlap 0 --launch-streams 0" "--overlap 0" ""; do
    timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 $F $v > $O/r06r_tmp.log 2>&1 || exit $?
    echo "$c [$v]: $(tail -1 $O/r06r_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["launch_streams"])')" | tee -a $L
  done
done
CLI=raymarchrenderer_amd/rmr_cli
for m in "--per-sample" ""; do
  timeout -k 10 300 $CLI --scene scenes/cornell5.scene --size 1920x1080 --samples 64 --bounces 4 --out /tmp/cli.bmp $m > $O/r06r_cli_c2$m.log 2>&1 || exit $?
  echo "cli c2 [$m]: $(grep msamples $O/r06r_cli_c2$m.log)" | tee -a $L
done
