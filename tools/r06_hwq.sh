#!/bin/bash
# round 6: 8 hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) with two and three
# overlapping contexts, full bench lines
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06za_hwq.log; mkdir -p $O
for q in 4 8; do for ov in 1 2; do for c in c1 rm3 rm2; do
  st=30; [ $c = c1 ] && st=200; [ $c = rm2 ] && st=60
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --overlap $ov > $O/r06za_tmp.log 2>&1 || exit $?
  echo "hwq $q overlap $ov $c: $(tail -1 $O/r06za_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $L
done; done; done
