#!/bin/bash
# Round-4 A/B, eleventh part (diagnostic library): waves per SIMD of the approximate sphere/box kernel
# (Cornell-5; 6 = default, 7 = 72 VGPRs without spills) and of RM3 / the Mandelbulb.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run c2_waves $E --scenes cornell5 --rounds 5 --spp 64 RMR_JIT_OPTS -- "" "-DRMR_FAST_WAVES=7" || exit $?
run rm3_waves $E --scenes rm3 --rounds 6 --spp 4 RMR_JIT_OPTS -- "" "-DRMR_FAST_WAVES=7" "-DRMR_FAST_WAVES=6" || exit $?
exit 0
