#!/bin/bash
# Round-4 A/B, thirteenth part (diagnostic library): RM3 at 7 waves per SIMD — shading threshold,
# 64-unit chunks (1080p 4 spp, 16 bounces).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run rm3_shade_t7 $E --scenes rm3 --rounds 8 --spp 4 shade_t -- 16 20 24 12 || exit $?
run rm3_chunk7 $E --scenes rm3 --rounds 8 --spp 4 RMR_JIT_OPTS -- "" "-DRMR_CHUNK=64" || exit $?
exit 0
