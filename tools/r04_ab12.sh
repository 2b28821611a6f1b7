#!/bin/bash
# Round-4 A/B, twelfth part (diagnostic library): Cornell-5 at 7 waves per SIMD — shading and refill
# thresholds (1080p 64 spp).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run c2_shade_t7 $E --scenes cornell5 --rounds 4 --spp 64 shade_t -- 16 14 18 20 || exit $?
run c2_refill7 $E --scenes cornell5 --rounds 4 --spp 64 RMR_REFILL_T -- 8 4 6 12 || exit $?
exit 0
