#!/bin/bash
# Round-4 A/B, sixth part (diagnostic library): 64- against 128-unit work chunks with the partitioned
# work queue, every non-cache kernel class at its bench sample count.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run chunk_rm3 $E --scenes rm3 --rounds 6 --spp 4 RMR_JIT_OPTS -- "" "-DRMR_CHUNK=64" || exit $?
run chunk_c2 $E --scenes cornell5 --rounds 4 --spp 64 RMR_JIT_OPTS -- "" "-DRMR_CHUNK=64" || exit $?
run chunk_c3 $E --scenes mandelbulb --rounds 3 --spp 128 RMR_JIT_OPTS -- "" "-DRMR_CHUNK=64" || exit $?
run chunk_prog $E --scenes multilight,default,glass --rounds 3 --spp 16 RMR_JIT_OPTS -- "" "-DRMR_CHUNK=64" || exit $?
exit 0
