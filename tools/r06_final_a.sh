#!/bin/bash
# round-6 measurement set, part A: GPU suite, smoke, every bench config, the drop-in call pattern, the
# C++ device group
cd "$(dirname "$0")/.." || exit 2
TAG=${1:-r06z}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
bash tools/gpu_benchall.sh || exit $?
for c in c1 c2 c3 c4 c5 rm2 rm3; do cp gpurun_out/bench_$c.log gpurun_out/${TAG}_bench_$c.log; done
bash tools/api_render_probe.sh $TAG || exit $?
timeout -k 10 300 python bench.py --api group --gpus 1 --config c2 --steps 5 > gpurun_out/${TAG}_group_c2.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_group_c2.log | cut -c1-400
