#!/bin/bash
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_jit.py tests/test_host_cpp.py -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab.py raymarchrenderer_amd/librmr_base.so raymarchrenderer_amd/librmr.so --spp 16 --rounds 6 > gpurun_out/ab_r1j.log 2>&1 || exit $?
cat gpurun_out/ab_r1j.log
