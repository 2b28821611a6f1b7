#!/bin/bash
# round 6: with 8 hardware queues, the long frames (C2, C3) with two contexts, three contexts, and two
# contexts with launch slots
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06zb_hwq_long.log; mkdir -p $O
F="--no-cpu-baseline --no-psnr --no-count-pass"
for rep in 1 2; do for c in c2 c3; do
  st=4; [ $c = c3 ] && st=4
  for v in "--overlap 1" "--overlap 2" "--overlap 1 --launch-streams 2"; do
    timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 $F $v > $O/r06zb_tmp.log 2>&1 || exit $?
    echo "$c [$v]: $(tail -1 $O/r06zb_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $L
  done
done; done
