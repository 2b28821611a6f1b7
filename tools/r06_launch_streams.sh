#!/bin/bash
# round 6: launch slots (rmr_set_launch_streams): GPU tests, then bench lines with one context / two
# contexts, with and without slots, and the per-call drop-in pattern (call batching off)
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06p_launch_streams.log
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_calls.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/r06p_tests.log 2>&1; rc=$?
tail -12 $O/r06p_tests.log; [ $rc -eq 0 ] || exit $rc
F="--no-cpu-baseline --no-psnr --no-count-pass"
for c in c1 rm3 rm2 c2; do
  st=3; [ $c = c1 ] && st=200; [ $c = rm3 ] && st=30; [ $c = rm2 ] && st=60
  for v in "--overlap 1 --launch-streams 0" "--overlap 0 --launch-streams 0" "--overlap 0 --launch-streams 2" "--overlap 1 --launch-streams 2" "--overlap 0 --launch-streams 3"; do
    timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 $F $v > $O/r06p_tmp.log 2>&1 || exit $?
    echo "$c [$v]: $(tail -1 $O/r06p_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')" | tee -a $L
  done
done
for c in c2 rm3; do for ls in 0 2 3; do
  timeout -k 10 300 python bench.py --api render --config $c --steps 3 --warmup 1 --call-batching 0 --launch-streams $ls > $O/r06p_tmp.log 2>&1 || exit $?
  echo "api render $c cb0 ls$ls: $(tail -1 $O/r06p_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["calls"]["per_s"], d["bitwise_equal_to_batched"])')" | tee -a $L
done; done
