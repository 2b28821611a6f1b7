#!/bin/bash
# Round-4 A/B, seventh part (diagnostic library): C3 (Mandelbulb 1080p 128 spp) after the round's
# kernel changes — shading threshold, finishing-batch size, waves per SIMD.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run c3_shade_t $E --scenes mandelbulb --rounds 3 --spp 128 shade_t -- 4 8 12 16 || exit $?
run c3_fin $E --scenes mandelbulb --rounds 3 --spp 128 RMR_JIT_OPTS -- "" "-DRMR_MB_FIN=36" "-DRMR_MB_FIN=52" "-DRMR_MB_FIN=60" || exit $?
run c3_waves $E --scenes mandelbulb --rounds 3 --spp 128 RMR_JIT_OPTS -- "" "-DRMR_GENERAL_WAVES=7" "-DRMR_GENERAL_WAVES=6" || exit $?
exit 0
