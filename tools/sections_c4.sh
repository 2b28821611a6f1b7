#!/bin/bash
# Section cycles of the C4 cache kernel (RMR_PROFILE: [4] refill, [5] map() iterations, [6] shading,
# [7] total, [9] full map() batches inside [5]); csg256 at 1080p 8 spp, 4 bounces
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
RMR_JIT_OPTS=-DRMR_PROFILE timeout -k 10 120 python tools/stats_run.py --spp 8 --scene scenes/csg256.scene --bounces 4 > gpurun_out/sections_c4.log 2>&1 || exit $?
tail -1 gpurun_out/sections_c4.log
RMR_JIT_OPTS=-DRMR_GRID_STATS timeout -k 10 120 python tools/stats_run.py --spp 8 --scene scenes/csg256.scene --bounces 4 > gpurun_out/gridstats_c4.log 2>&1 || exit $?
tail -1 gpurun_out/gridstats_c4.log
