cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 tools/probes/sqrt_exhaustive > gpurun_out/sqrt_exhaustive.log 2>&1; echo "sqrt rc=$?"
timeout -k 10 600 python -m pytest tests -m gpu -q -s > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/tune.py --configs '[{"T":8},{"T":10},{"T":12},{"T":16}]' > gpurun_out/tune3.log 2>&1
