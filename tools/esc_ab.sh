#!/bin/bash
# The escape bound for every kernel class (round 3: RM2 incl. shadow rays, node-program-material
# kernels): tools/librmr_base.so (HO kernels only) against the working tree, same process, bitwise.
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
: > gpurun_out/esc_ab.log
G=tests/golden/scenes
for spec in "$G/simple.scene 2 16" "$G/default.scene 1 8" "$G/glass_test.scene 1 8" "$G/multilight.scene 1 8"; do
  set -- $spec
  echo "scene $1 variant $2 bounces $3" >> gpurun_out/esc_ab.log
  timeout -k 10 300 python tools/ab.py tools/librmr_base.so raymarchrenderer_amd/librmr.so --scene $1 --variant $2 --bounces $3 --spp 16 --rounds 5 >> gpurun_out/esc_ab.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/esc_ab.log
