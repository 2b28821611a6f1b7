#!/bin/bash
# round 6: short frames with 3 (kept) / 4 / 5 overlapping contexts, 8 hardware queues
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06zc_ctx45.log; mkdir -p $O
F="--no-cpu-baseline --no-psnr --no-count-pass"
for c in c1 rm2 rm3; do
  st=30; [ $c = c1 ] && st=200; [ $c = rm2 ] && st=60
  for v in 2 3 4; do
    timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 $F --overlap $v > $O/r06zc_tmp.log 2>&1 || exit $?
    echo "$c [overlap $v]: $(tail -1 $O/r06zc_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $L
  done
done
