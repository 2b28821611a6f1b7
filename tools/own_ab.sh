#!/bin/bash
# Pixel-owned units (RMR_OWN) against per-sample units + k_fold: same process, bitwise compared;
# the per-sample tail at 0.5 / 1 / 2 x the grid's lanes (RMR_OWN_TAIL).
set -o pipefail
mkdir -p gpurun_out
for tail in 1 0.5 2; do
  RMR_OWN_TAIL=$tail timeout -k 10 400 python tools/env_ab.py RMR_JIT_OPTS --scenes cornell5,mandelbulb,csg256,rm3 --spp 64 --rounds 3 -- " " "-DRMR_OWN" > gpurun_out/own_ab_$tail.log 2>&1 || exit $?
  echo "tail $tail"; cat gpurun_out/own_ab_$tail.log | grep scene
done
