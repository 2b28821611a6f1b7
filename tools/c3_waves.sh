#!/bin/bash
# C3 (Mandelbulb, 1080p 128 spp): waves per SIMD of the general-map kernel, same process, bitwise.
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/env_ab.py RMR_JIT_OPTS --scenes mandelbulb --spp 128 --rounds 5 -- " " "-DRMR_GENERAL_WAVES=7" "-DRMR_GENERAL_WAVES=6" > gpurun_out/c3_waves.log 2>&1 || exit $?
grep scene gpurun_out/c3_waves.log
