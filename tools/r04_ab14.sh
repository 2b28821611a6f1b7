#!/bin/bash
# Round-4 A/B, fourteenth part (diagnostic library): the stepped Mandelbulb map with two estimator
# iterations per pass (an RMR_MB_PASS option, removed again after this measurement: +1.2%)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
timeout -k 10 500 python -u tools/env_ab.py --scenes mandelbulb --rounds 4 --spp 128 RMR_JIT_OPTS -- "" "-DRMR_MB_PASS=2" "-DRMR_MB_PASS=2 -DRMR_MB_FIN=36" > gpurun_out/r04ab_c3_pass2.log 2>&1 || exit $?
tail -2 gpurun_out/r04ab_c3_pass2.log
