cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_calls.py tests/test_gpu_group.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r06c_tests.log 2>&1; rc=$?; tail -15 gpurun_out/r06c_tests.log; [ $rc -le 1 ] || exit $rc
for c in c2 rm3; do timeout -k 10 300 python bench.py --api group --gpus 1 --config $c --steps 3 > gpurun_out/r06c_group_$c.log 2>&1 || exit $?; tail -1 gpurun_out/r06c_group_$c.log | cut -c1-1200; done
