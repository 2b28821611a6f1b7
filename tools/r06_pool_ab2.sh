#!/bin/bash
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python tools/abrun.py --cases c4,csg64 --rounds 3 nopool="opts:-DRMR_NPC_POOL=0" p5nr="opts:-DRMR_CACHE_WAVES=5 -DRMR_POOL_RATIO=0" p5nrns="opts:-DRMR_CACHE_WAVES=5 -DRMR_POOL_RATIO=0 -DRMR_POOL_SLEEP=0" p5s40="opts:-DRMR_CACHE_WAVES=5 -DRMR_POOL_RATIO=0 -DRMR_POOL_SERVE=40" > $O/r06h_pool_ab2.log 2>&1 || exit $?
grep '"case"' $O/r06h_pool_ab2.log | cut -c1-2400
timeout -k 10 300 python tools/abrun.py --cases c4 --rounds 2 p5nr="opts:-DRMR_CACHE_WAVES=5 -DRMR_POOL_RATIO=0 -DRMR_PROFILE" > $O/r06h_pool_sections2.log 2>&1 || exit $?
grep '"case"' $O/r06h_pool_sections2.log | cut -c1-2400
