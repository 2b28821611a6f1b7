#!/bin/bash
# Round-4 A/B, ninth part (diagnostic library): the escape boxes of small scenes (one per primitive)
# against their bounding box alone (RMR_ESC_MERGE=1).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run merge_c2 $E --scenes cornell5 --rounds 4 --spp 64 RMR_ESC_MERGE -- 0 1 || exit $?
run merge_rm $E --scenes rm3,rm2simple --rounds 6 --spp 4 RMR_ESC_MERGE -- 0 1 || exit $?
run merge_c3 $E --scenes mandelbulb --rounds 3 --spp 128 RMR_ESC_MERGE -- 0 1 || exit $?
run merge_prog $E --scenes multilight,default,glass --rounds 3 --spp 16 RMR_ESC_MERGE -- 0 1 || exit $?
exit 0
