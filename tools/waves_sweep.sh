#!/bin/bash
# Occupancy / scheduler sweeps of the specialised kernels (RMR_JIT_OPTS / RMR_JIT_SCHED are part of the
# code-object key, so one process compiles each variant): csg256 (cache kernels), Mandelbulb, RM3
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python tools/env_ab.py RMR_JIT_OPTS --scenes csg256 --spp 8 --rounds 3 -- " " "-DRMR_CACHE_WAVES=5" "-DRMR_CACHE_WAVES=7" > gpurun_out/w_c4.log 2>&1 || exit $?
cat gpurun_out/w_c4.log
timeout -k 10 400 python tools/env_ab.py RMR_JIT_SCHED 1 0 --scenes csg256 --spp 8 --rounds 3 > gpurun_out/w_c4s.log 2>&1 || exit $?
cat gpurun_out/w_c4s.log
timeout -k 10 400 python tools/env_ab.py RMR_JIT_OPTS --scenes mandelbulb --spp 16 --rounds 3 -- " " "-DRMR_GENERAL_WAVES=6" "-DRMR_GENERAL_WAVES=7" > gpurun_out/w_c3.log 2>&1 || exit $?
cat gpurun_out/w_c3.log
timeout -k 10 400 python tools/env_ab.py RMR_JIT_OPTS --scenes rm3 --spp 16 --rounds 3 -- " " "-DRMR_FAST_WAVES=6" "-DRMR_FAST_WAVES=7" > gpurun_out/w_rm3.log 2>&1 || exit $?
cat gpurun_out/w_rm3.log
