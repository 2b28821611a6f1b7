#!/bin/bash
# parity (no -x: see every failure) + A/B of the lane-state diet + bench line
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab.py raymarchrenderer_amd/librmr_base.so raymarchrenderer_amd/librmr.so raymarchrenderer_amd/librmr_w10.so raymarchrenderer_amd/librmr_w6.so --spp 8 --rounds 6 > gpurun_out/ab_r1a.log 2>&1 || exit $?
cat gpurun_out/ab_r1a.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1a.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r1a.log | cut -c1-400
