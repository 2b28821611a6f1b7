#!/bin/bash
cd "$(dirname "$0")/.." || exit 2
timeout -k 10 300 python tools/ab.py raymarchrenderer_amd/librmr.so raymarchrenderer_amd/librmr_expcornell.so --spp 16 --rounds 6 --T $((16 | (4 << 8))) > gpurun_out/ab_r1e.log 2>&1 || exit $?
cat gpurun_out/ab_r1e.log
timeout -k 10 300 python tools/ab.py raymarchrenderer_amd/librmr.so raymarchrenderer_amd/librmr_expcornell.so --spp 16 --rounds 6 > gpurun_out/ab_r1e2.log 2>&1 || exit $?
cat gpurun_out/ab_r1e2.log
