#!/bin/bash
# Renderer contexts per process (bench.py --overlap K: K + 1 contexts on as many streams), round 4:
# RM3 / RM2 / C1 / C2 bench lines at K = 1 (default), 2, 3; two rounds.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
for i in 1 2; do
for k in 1 2 3; do
  for c in rm3 rm2 c1 c2; do
    st=30; [ $c = rm2 ] && st=60; [ $c = c1 ] && st=200; [ $c = c2 ] && st=10
    timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 --overlap $k --no-cpu-baseline --no-psnr --no-count-pass > gpurun_out/ovl_$c.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ovl_$c.log').read().strip().splitlines()[-1]);print('$c', 'overlap $k', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done; done
