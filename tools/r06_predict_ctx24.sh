#!/bin/bash
# round 6: the 2- and 4-rank C2 shares' predictions with 2 / 4 overlapping contexts (8 hardware queues)
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06zh_predict_ctx24.log; mkdir -p $O
for v in 1 3; do
  timeout -k 10 400 python bench.py --config c2 --predict 2,4 --steps 8 --warmup 2 --overlap $v > $O/r06zh_tmp.log 2>&1 || exit $?
  echo "predict c2 [overlap $v]: $(tail -1 $O/r06zh_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["partition_prediction"]; t=d["tiles"]["32"]; print({n: (t[n]["rank_ms"][:2], t[n]["predicted_speedup"]) for n in ("2","4")}, d["one_gpu_ms"])')" | tee -a $L
done
