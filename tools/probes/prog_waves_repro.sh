#!/bin/bash
# Reproducer of the forced-wave node-program miscompile (profiles/r04_prog_waves_diag.md).
#
# CPU part (this container): dump glass_test.scene's generated kernel source through the diagnostic
# library, compile it with hipcc at the allocator's wave target and with -DRMR_PROG_WAVES=7, and
# print each build's VGPR / spill / scratch notes. With the extra hipcc words in $EXTRA (e.g.
# "-mllvm -amdgpu-opt-vgpr-liverange=false") the forced build is compiled with them as well.
#
# GPU part (--gpu, on the box): tools/prog_waves_diag.py renders glass_test with the default and the
# forced builds and counts the samples that differ bitwise (6469 / 5774 of 98304 at 6 / 7 waves, 0
# with SIOptimizeVGPRLiveRange disabled).
#
#   tools/probes/prog_waves_repro.sh [--gpu]
set -e
cd "$(dirname "$0")/../.."
OUT=${OUT:-/tmp/prog_waves_repro}
mkdir -p "$OUT"
if [ "$1" = --gpu ]; then
  python -u tools/prog_waves_diag.py --waves 6,7; exit $?
fi
rm -f "$OUT"/*.hip
RMR_LIB=diag RMR_JIT_DUMP="$OUT" RMR_JIT_CACHE="$OUT/cache" python - <<'EOF'
from raymarchrenderer_amd import renderer as rmr
rmr.jit_compile_scene("tests/golden/scenes/glass_test.scene", "rm1", diag=True)
EOF
SRC=$(ls -t "$OUT"/*.hip | head -n 1)
# the hipRTC options of rmr_jit.cpp (kOptions) and the source's own //@opts lines
OPTS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Wno-unused-function -fno-slp-vectorize -DRMR_MANDELBULB_INLINE=1"
OPTS="$OPTS $(grep '^//@opts ' "$SRC" | sed 's|^//@opts ||' | tr '\n' ' ')"
notes() {   # name, extra options...
  local n=$1; shift
  hipcc $OPTS "$@" -I raymarchrenderer_amd/csrc --offload-device-only --no-gpu-bundle-output -c -o "$OUT/$n.o" -x hip "$SRC"
  echo "== $n ($*)"
  /opt/rocm/lib/llvm/bin/llvm-readelf --notes "$OUT/$n.o" |
    grep -E '\.(vgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size):' | sort -u
}
notes default
notes waves7 -DRMR_PROG_WAVES=7
[ -n "$EXTRA" ] && notes waves7_extra -DRMR_PROG_WAVES=7 $EXTRA
echo "source: $SRC"
