#!/bin/bash
# One GPU session: parity tests, smoke, short bench. Stops at the first crash/timeout
# (exit 124/134/137/139); a plain test failure (exit 1) still lets the bench run.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 ${T_TEST:-420} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=20 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?
echo "smoke rc=$rc2"; tail -3 gpurun_out/smoke.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 ${T_BENCH:-300} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc3=$?
echo "bench rc=$rc3"; tail -3 gpurun_out/bench.log
exit $rc3
