#!/bin/bash
# Same-process A/B of LLVM machine-scheduler options for the hipRTC kernels (RMR_JIT_OPTS).
# " -DRMR_AB_DUP=1" (an unused macro) builds the default kernel under another code-object key: the
# baseline again, run last in each round. OPTS overrides the option sets (one per line).
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
mkdir -p gpurun_out
DEF=$'-mllvm --amdgpu-sched-strategy=max-memory-clause\n-mllvm --amdgpu-sched-strategy=iterative-ilp\n-mllvm --amdgpu-sched-strategy=max-ilp'
mapfile -t SETS <<< "${OPTS:-$DEF}"
timeout -k 10 500 python -u tools/env_ab.py --scenes ${SCENES:-cornell5,rm3,mandelbulb,default,multilight} --spp ${SPP:-64} --rounds ${ROUNDS:-5} RMR_JIT_OPTS "" "${SETS[@]}" " -DRMR_AB_DUP=1" > gpurun_out/sched_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/sched_ab.log | tail -20; exit $rc
