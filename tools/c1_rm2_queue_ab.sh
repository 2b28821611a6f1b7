#!/bin/bash
# Same-box A/B of the work queue's variants on the short-frame configs (C1, RM2) through bench.py
# (diagnostic library, RMR_JIT_OPTS), two rounds.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
for i in 1 2; do
for v in "" "-DRMR_QUEUE_SEQ=16"; do
  for c in c1 rm2; do
    st=200; [ $c = rm2 ] && st=60
    RMR_LIB=diag RMR_JIT_OPTS="$v" timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline --no-psnr --no-count-pass > gpurun_out/qab_$c.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/qab_$c.log').read().strip().splitlines()[-1]);print('$c', repr('$v'), d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done; done
