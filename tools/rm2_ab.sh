#!/bin/bash
# RM2 (simple.scene, 1080p 16 spp 16 bounces): the previous revision's library (tools/librmr_base.so,
# v2 material interpreted from the tables) against the working tree's (straight-line JitV2Mats), same
# process. Bitwise compared. (Measured once as well: 6 / 8 waves per SIMD for the RM2 kernel instead of
# the allocator's choice, 3.23 / 3.35 against 3.18 ms.)
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab.py tools/librmr_base.so raymarchrenderer_amd/librmr.so --scene tests/golden/scenes/simple.scene --variant 2 --bounces 16 --spp 16 --rounds 6 > gpurun_out/rm2_ab.log 2>&1 || exit $?
cat gpurun_out/rm2_ab.log
