#!/bin/bash
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_jit.py -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/tune.py --spp 16 --configs '[{"T":16,"TR":8},{"T":16,"TR":4},{"T":16,"TR":2},{"T":16,"TR":1},{"T":12,"TR":2},{"T":20,"TR":2},{"T":16,"TR":8},{"T":16,"TR":2}]' > gpurun_out/tune_lds.log 2>&1 || exit $?
cut -c1-150 gpurun_out/tune_lds.log
