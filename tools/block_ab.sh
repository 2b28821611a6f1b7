#!/bin/bash
# Threads per block of the specialised trace kernel (a diagnostic RMR_JIT_BLOCK option, removed again after this
# measurement, profiles/r04_block_ab.log): 256 / 128 / 64
# through bench.py (two overlapping renderer contexts), two rounds; short-frame configs first.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
for i in 1 2; do
for b in 256 128 64; do
  for c in rm3 rm2 c1 c2 c3; do
    st=30; [ $c = rm2 ] && st=60; [ $c = c1 ] && st=200; [ $c = c2 ] && st=10; [ $c = c3 ] && st=5
    RMR_LIB=diag RMR_JIT_BLOCK=$b timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline --no-psnr --no-count-pass > gpurun_out/blk_$c.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/blk_$c.log').read().strip().splitlines()[-1]);print('$c', 'block $b', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done; done
