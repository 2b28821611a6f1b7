#!/bin/bash
# round 6: the per-call drop-in loop (call batching off) with 2 (default) / 3 / 4 launch slots, under
# bench.py's 8 hardware queues
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06ze_api_ls.log; mkdir -p $O
for c in c2 rm3; do for ls in 2 3 4; do
  timeout -k 10 300 python bench.py --api render --config $c --steps 3 --warmup 1 --call-batching 0 --launch-streams $ls > $O/r06ze_tmp.log 2>&1 || exit $?
  echo "api render $c cb0 ls$ls: $(tail -1 $O/r06ze_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["calls"]["per_s"], d["bitwise_equal_to_batched"])')" | tee -a $L
done; done
