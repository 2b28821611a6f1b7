#!/bin/bash
# round 6: one context on a caller's (torch) stream with launch slots re-created after rmr_set_stream
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; L=$O/r06v_set_stream_slots.log; mkdir -p $O
F="--no-cpu-baseline --no-psnr --no-count-pass"
for c in c1 rm3 rm2; do
  st=30; [ $c = c1 ] && st=200; [ $c = rm2 ] && st=60
  for v in "--overlap 0 --launch-streams 0" "--overlap 0" ""; do
    timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 $F $v > $O/r06v_tmp.log 2>&1 || exit $?
    echo "$c [$v]: $(tail -1 $O/r06v_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["launch_streams"])')" | tee -a $L
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_calls.py tests/test_multi_gpu_cpu.py tests/test_gpu_coverage.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r06v_tests.log 2>&1; rc=$?; tail -2 $O/r06v_tests.log; exit $rc
