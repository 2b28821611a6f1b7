#!/bin/bash
# Primary rays' first march step from one map(eye) per wave (RMR_CULL_EYE, culling 15) against the
# per-lane step (culling 7), every scene family of tools/env_ab.py, same process, bitwise check;
# then the GPU test suite
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 500 python tools/env_ab.py --spp ${SPP:-16} --rounds ${ROUNDS:-5} ${SCENES:+--scenes $SCENES} culling 7 15 > gpurun_out/eye_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/eye_ab.log
[ -n "$NOTEST" ] && exit 0
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; exit $rc
