#!/bin/bash
# Round-4 A/B, third part: the GPU suite on the release library, then (diagnostic library) the work
# queue's partitions (1 = one counter, the round-3 queue) and the RM1 shading threshold.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ab_gpu_tests3.log 2>&1 || { tail -30 gpurun_out/r04ab_gpu_tests3.log; exit 1; }
tail -2 gpurun_out/r04ab_gpu_tests3.log
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run parts $E --scenes rm2simple,rm3,cornell5,mandelbulb,multilight --rounds 4 --spp 16 RMR_JIT_OPTS -- "" "-DRMR_QUEUE_PARTS=1" "-DRMR_QUEUE_PARTS=4" "-DRMR_QUEUE_PARTS=16" || exit $?
run parts_c4 $E --scenes csg256 --rounds 3 --spp 8 RMR_JIT_OPTS -- "" "-DRMR_QUEUE_PARTS=1" || exit $?
run shade_t $E --scenes cornell5,multilight,default,rm3 --rounds 3 --spp 16 shade_t -- 16 20 24 32 || exit $?
exit 0
