#!/bin/bash
# Round-4 A/B, seventeenth part (diagnostic library): Cornell-5 refill threshold with 20-lane shading
# batches (default refill: half the shading threshold, 10).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
timeout -k 10 500 python -u tools/env_ab.py --scenes cornell5 --rounds 5 --spp 64 RMR_REFILL_T -- 10 6 8 14 > gpurun_out/r04ab_c2_refill20.log 2>&1 || exit $?
tail -1 gpurun_out/r04ab_c2_refill20.log
