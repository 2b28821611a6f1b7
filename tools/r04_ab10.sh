#!/bin/bash
# Round-4 A/B, tenth part (diagnostic library): C4's full-batch threshold / ratio, shading threshold
# and refill threshold after the round's changes (csg256 1080p 8 spp).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run c4_full_t $E --scenes csg256 --rounds 3 --spp 8 RMR_FULL_T -- 40 32 48 56 || exit $?
run c4_full_r $E --scenes csg256 --rounds 3 --spp 8 RMR_FULL_R -- 8 4 12 16 || exit $?
run c4_shade_t $E --scenes csg256 --rounds 3 --spp 8 shade_t -- 16 12 20 24 || exit $?
run c4_refill $E --scenes csg256 --rounds 3 --spp 8 RMR_REFILL_T -- 8 4 12 16 || exit $?
exit 0
