#!/bin/bash
# Round-4 A/B, eighth part (diagnostic library): the escape bound on / off per kernel class (culling
# 15 = all, 14 = all but RMR_CULL_ESCAPE) at the bench sample counts.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run esc_c2 $E --scenes cornell5 --rounds 4 --spp 64 culling -- 15 14 || exit $?
run esc_rm3 $E --scenes rm3,rm2simple --rounds 6 --spp 4 culling -- 15 14 || exit $?
run esc_c3 $E --scenes mandelbulb --rounds 3 --spp 128 culling -- 15 14 || exit $?
run esc_prog $E --scenes multilight,default,glass --rounds 3 --spp 16 culling -- 15 14 || exit $?
exit 0
