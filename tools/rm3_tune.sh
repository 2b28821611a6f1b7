#!/bin/bash
# RM3 as wired (built-in spectral scene, 16 bounces): shading-batch threshold sweep (refill at half
# of it), same process, bitwise compared. 1080p 16 spp.
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python tools/env_ab.py shade_t 16 8 12 24 32 --scenes rm3 --spp 16 --rounds 4 > gpurun_out/rm3_tune.log 2>&1 || exit $?
grep scene gpurun_out/rm3_tune.log
timeout -k 10 300 python tools/env_ab.py shade_t 16 8 12 24 32 --scenes rm2simple --spp 16 --rounds 4 >> gpurun_out/rm3_tune.log 2>&1 || exit $?
grep scene gpurun_out/rm3_tune.log | tail -1
