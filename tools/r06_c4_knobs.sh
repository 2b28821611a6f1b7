#!/bin/bash
# round 6: the cache kernel's full-batch thresholds and cache size after the SoA table
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python tools/abrun.py --cases c4,csg64 --rounds 3 def="" t32="env:RMR_FULL_T=32" t48="env:RMR_FULL_T=48" r4="env:RMR_FULL_R=4" r16="env:RMR_FULL_R=16" k1="opts:-DRMR_NPC_K=1" > $O/r06j_c4_knobs.log 2>&1 || exit $?
grep '"case"' $O/r06j_c4_knobs.log | cut -c1-3000
