#!/bin/bash
# Round-4 A/B, fourth part (diagnostic library): work-queue partitions 16 / 32 / 64, RM2 / C1 / C4 too;
# the node-program kernels' shading threshold on glass.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run parts2 $E --scenes rm2simple,rm3,cornell5,mandelbulb --rounds 4 --spp 16 RMR_JIT_OPTS -- "" "-DRMR_QUEUE_PARTS=32" "-DRMR_QUEUE_PARTS=64" || exit $?
run parts2_rm2_4spp $E --scenes rm2simple --rounds 6 --spp 4 RMR_JIT_OPTS -- "" "-DRMR_QUEUE_PARTS=8" "-DRMR_QUEUE_PARTS=32" "-DRMR_QUEUE_PARTS=64" || exit $?
run parts2_c4 $E --scenes csg256 --rounds 3 --spp 8 RMR_JIT_OPTS -- "" "-DRMR_QUEUE_PARTS=64" || exit $?
run shade_t_glass $E --scenes glass,multilight,default --rounds 3 --spp 16 shade_t -- 16 20 || exit $?
exit 0
