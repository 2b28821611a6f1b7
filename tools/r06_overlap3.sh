#!/bin/bash
# round 6: three overlapping contexts (3 streams + torch's default: within the 4 hardware queues)
# against two, on the N = 1 line and the 8-rank share prediction
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06z8_overlap3.log; mkdir -p $O
F="--no-cpu-baseline --no-psnr --no-count-pass"
for c in rm3 c1 rm2 c2; do
  st=30; [ $c = c1 ] && st=200; [ $c = rm2 ] && st=60; [ $c = c2 ] && st=4
  for v in "--overlap 1" "--overlap 2"; do
    timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 $F $v > $O/r06z8_tmp.log 2>&1 || exit $?
    echo "$c [$v]: $(tail -1 $O/r06z8_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $L
  done
done
for v in "--overlap 1" "--overlap 2"; do
  timeout -k 10 300 python bench.py --config c2 --predict 8 --steps 16 --warmup 2 $v > $O/r06z8_tmp.log 2>&1 || exit $?
  echo "predict c2 8 [$v]: $(tail -1 $O/r06z8_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["partition_prediction"]; t=d["tiles"]["32"]["8"]; print(t["predicted_speedup"], t["max_over_mean"], d["one_gpu_ms"])')" | tee -a $L
done
