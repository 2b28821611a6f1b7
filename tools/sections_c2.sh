#!/bin/bash
# Section cycles of the specialised kernel (RMR_PROFILE build: counters [4] refill / ray setup,
# [5] map() iterations, [6] shading batches, [7] total, summed over waves) for C2 and C3.
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
RMR_JIT_OPTS=-DRMR_PROFILE timeout -k 10 120 python tools/stats_run.py --spp 16 > gpurun_out/sections_c2.log 2>&1 || exit $?
tail -1 gpurun_out/sections_c2.log
RMR_JIT_OPTS=-DRMR_PROFILE timeout -k 10 120 python tools/stats_run.py --spp 16 --scene scenes/mandelbulb.scene --bounces 2 > gpurun_out/sections_c3.log 2>&1 || exit $?
tail -1 gpurun_out/sections_c3.log
