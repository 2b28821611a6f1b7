#!/bin/bash
# Round-4 A/B, fifteenth part (diagnostic library): the certified kernels' primitive table in LDS for
# cert_normals (an RMR_CERT_LDS option, removed again after this measurement: -0.24%, within noise)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
timeout -k 10 500 python -u tools/env_ab.py --scenes cornell5 --rounds 6 --spp 64 RMR_JIT_OPTS -- "" "-DRMR_CERT_LDS=0" > gpurun_out/r04ab_c2_certlds.log 2>&1 || exit $?
tail -1 gpurun_out/r04ab_c2_certlds.log
