#!/bin/bash
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log; grep "PSNR" gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -m pytest tests/test_gpu_reference_psnr.py -m gpu -q -s > gpurun_out/psnr.log 2>&1; grep PSNR gpurun_out/psnr.log
timeout -k 10 300 python tools/ab.py raymarchrenderer_amd/librmr_base.so raymarchrenderer_amd/librmr.so --spp 8 --rounds 6 > gpurun_out/ab_r1b.log 2>&1 || exit $?
cat gpurun_out/ab_r1b.log
timeout -k 10 300 python bench.py > gpurun_out/bench_r1b.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r1b.log | cut -c1-300
for c in c3 c1; do timeout -k 10 300 python bench.py --config $c --steps 2 > gpurun_out/bench_r1b_$c.log 2>&1 || exit $?; tail -1 gpurun_out/bench_r1b_$c.log | cut -c1-250; done
