#!/bin/bash
# N = 1: one renderer context against two / three overlapping ones (consecutive frames on separate
# streams), per config; 10 timed steps each, no side legs.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/overlap_ab.log
for cfg in rm3 rm2 c1 c2 c3; do
  for ov in 0 1 2; do
    st=10; [ $cfg = c1 ] && st=200; [ $cfg = rm2 ] && st=40; [ $cfg = rm3 ] && st=30
    timeout -k 10 200 python bench.py --config $cfg --overlap $ov --steps $st --warmup 3 --no-psnr --no-cpu-baseline --no-count-pass > gpurun_out/ov.json 2>/dev/null || exit $?
    python -c "
import json,sys; d=json.loads(open('gpurun_out/ov.json').read().strip().splitlines()[-1])
print(json.dumps({'config':'$cfg','overlap':$ov,'value':d['value'],'ms_per_step':d['ms_per_step'],'avg_launch_ms':d['roofline']['avg_launch_ms']}))" | tee -a gpurun_out/overlap_ab.log
  done
done
