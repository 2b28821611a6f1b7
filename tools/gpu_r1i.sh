#!/bin/bash
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -m pytest tests/test_gpu_reference_psnr.py -m gpu -q -s > gpurun_out/psnr.log 2>&1; grep PSNR gpurun_out/psnr.log
exit $rc
