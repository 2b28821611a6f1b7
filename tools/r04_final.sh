#!/bin/bash
# Round-4 end: the GPU suite on the release library, then tools/r04_final_prof.sh (HEAD profiles of
# every bench config, tags r04z_<config>).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04z_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04z_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04z_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04z_smoke.log 2>&1 || { tail -20 gpurun_out/r04z_smoke.log; exit 1; }
tail -2 gpurun_out/r04z_smoke.log
bash tools/r04_final_prof.sh
