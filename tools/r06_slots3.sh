#!/bin/bash
# round 6: one context with 2 / 3 / 4 launch slots against the default two contexts (frame path)
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06x_slots_n.log; mkdir -p $O
F="--no-cpu-baseline --no-psnr --no-count-pass"
for c in rm3 c1 rm2 c2; do
  st=30; [ $c = c1 ] && st=200; [ $c = rm2 ] && st=60; [ $c = c2 ] && st=3
  for v in "" "--overlap 0 --launch-streams 2" "--overlap 0 --launch-streams 3" "--overlap 0 --launch-streams 4"; do
    timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 $F $v > $O/r06x_tmp.log 2>&1 || exit $?
    echo "$c [$v]: $(tail -1 $O/r06x_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["launch_streams"])')" | tee -a $L
  done
done
