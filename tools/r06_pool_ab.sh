#!/bin/bash
# round 6: the block pool of full map() requests (C4 cache kernel) against the kernel without it
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python tools/abrun.py --cases c4,csg64 --rounds 3 nopool="opts:-DRMR_NPC_POOL=0" pool6="" pool5="opts:-DRMR_CACHE_WAVES=5" pool5c64="opts:-DRMR_CACHE_WAVES=5 -DRMR_CHUNK_POOL=64" pool5s48="opts:-DRMR_CACHE_WAVES=5 -DRMR_POOL_SERVE=48" > $O/r06g_pool_ab.log 2>&1 || exit $?
grep '"case"' $O/r06g_pool_ab.log | cut -c1-2400
timeout -k 10 300 python tools/abrun.py --cases c4 --rounds 2 nopool="opts:-DRMR_NPC_POOL=0 -DRMR_PROFILE" pool6="opts:-DRMR_PROFILE" pool5="opts:-DRMR_CACHE_WAVES=5 -DRMR_PROFILE" > $O/r06g_pool_sections.log 2>&1 || exit $?
grep '"case"' $O/r06g_pool_sections.log | cut -c1-2400
echo done
