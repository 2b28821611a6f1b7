#!/bin/bash
# C3 (Mandelbulb): the stepped map (finishing batches of RMR_MB_FIN lanes) against the whole map per
# pass (-DRMR_MB_STEPPED=0), finishing-batch sizes and waves per SIMD, same process; then the
# Mandelbulb GPU parity tests
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
A="--scenes mandelbulb --spp ${SPP:-32} --rounds ${ROUNDS:-5}"
timeout -k 10 400 python tools/env_ab.py $A RMR_JIT_OPTS -- ${OPTS:-"-DRMR_MB_STEPPED=0" "-DRMR_MB_FIN=24" "-DRMR_MB_FIN=28" "-DRMR_MB_FIN=32" "-DRMR_MB_FIN=36" "-DRMR_MB_FIN=44" "-DRMR_MB_STEPPED=0"} > gpurun_out/c3_fin.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/c3_fin.log
