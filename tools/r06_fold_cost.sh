#!/bin/bash
# round 6: the headline bench with and without the k_fold launch (diagnostic library,
# RMR_DIAG_NO_FOLD=1: timing only, wrong accumulator): the ceiling of folding inside the trace kernel.
# Alternating runs, C2 and RM2 (the config where the fold is the largest share of a frame)
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out
export RMR_LIB=diag
for i in 1 2 3; do
  for nf in 0 1; do
    for c in c2 rm2; do
      st=5; [ $c = rm2 ] && st=60
      RMR_DIAG_NO_FOLD=$nf timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline --no-psnr --no-count-pass > $O/r06n_fold_${c}_nf${nf}_$i.log 2>&1 || exit $?
      echo "$c nofold=$nf run $i: $(tail -1 $O/r06n_fold_${c}_nf${nf}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')" | tee -a $O/r06n_fold_cost.log
    done
  done
done
