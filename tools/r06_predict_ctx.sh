#!/bin/bash
# round 6: the 8-rank C2 share's prediction with 2 / 3 / 4 overlapping contexts (8 hardware queues)
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06zd_predict_ctx.log; mkdir -p $O
for v in 1 2 3; do
  timeout -k 10 300 python bench.py --config c2 --predict 8 --steps 16 --warmup 2 --overlap $v > $O/r06zd_tmp.log 2>&1 || exit $?
  echo "predict c2 8 [overlap $v]: $(tail -1 $O/r06zd_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["partition_prediction"]; t=d["tiles"]["32"]["8"]; print(t["predicted_speedup"], t["max_over_mean"], t["rank_ms"][:2], d["one_gpu_ms"])')" | tee -a $L
done
