#!/bin/bash
# Same-process A/B of tools/librmr_base.so (a previous revision, tools/build_rev.sh) against the
# working tree's librmr.so on csg256 (C4's scene) and Cornell-5; bitwise comparison included
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab.py tools/librmr_base.so raymarchrenderer_amd/librmr.so --scene scenes/csg256.scene --spp 8 --rounds 6 > gpurun_out/ab_c4.log 2>&1 || exit $?
cat gpurun_out/ab_c4.log
