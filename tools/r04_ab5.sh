#!/bin/bash
# Round-4 A/B, fifth part (diagnostic library): RM2 after the partitioned work queue — light-side
# shadow bound, wave target, shading threshold; RM3 shading threshold.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run rm2_light2 $E --scenes rm2simple --rounds 8 --spp 4 RMR_JIT_OPTS -- "" "-DRMR_SHADOW_LIGHT_BOUND=0" || exit $?
run rm2_waves2 $E --scenes rm2simple --rounds 6 --spp 4 RMR_JIT_OPTS -- "" "-DRMR_RM2_WAVES=5" "-DRMR_RM2_WAVES=7" "-DRMR_RM2_WAVES=8" || exit $?
run rm2_shade_t $E --scenes rm2simple --rounds 6 --spp 4 shade_t -- 12 16 24 32 || exit $?
run rm3_chunk $E --scenes rm3,rm2simple --rounds 4 --spp 4 RMR_JIT_OPTS -- "" "-DRMR_CHUNK=64" || exit $?
exit 0
