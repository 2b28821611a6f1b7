#!/bin/bash
# Round-4 A/B, sixteenth part (diagnostic library): tile-major work order (an RMR_TILE_MAJOR option, removed
# again after this measurement; a chunk was one tile's consecutive samples, a queue partition a band of tiles)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 500 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -8
}
E="python -u tools/env_ab.py"
run tm_c4 $E --scenes csg256 --rounds 3 --spp 32 RMR_JIT_OPTS -- "" "-DRMR_TILE_MAJOR=1" || exit $?
run tm_c2 $E --scenes cornell5,mandelbulb --rounds 3 --spp 64 RMR_JIT_OPTS -- "" "-DRMR_TILE_MAJOR=1" || exit $?
run tm_rm $E --scenes rm3,rm2simple,multilight --rounds 4 --spp 4 RMR_JIT_OPTS -- "" "-DRMR_TILE_MAJOR=1" || exit $?
exit 0
