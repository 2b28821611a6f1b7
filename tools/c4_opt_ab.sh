#!/bin/bash
# C4 cache kernel: same-process A/B of compile-time switches (OPTS: RMR_JIT_OPTS values) on csg256,
# bitwise check; then the csg / grid / culling GPU tests
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python tools/env_ab.py --scenes csg256 --spp ${SPP:-8} --rounds ${ROUNDS:-6} RMR_JIT_OPTS -- ${OPTS} > gpurun_out/c4_opt.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/c4_opt.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "csg or bvh or grid or culling or coverage" > gpurun_out/pytest_c4.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_c4.log; exit $rc
