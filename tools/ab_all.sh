#!/bin/bash
# Same-process A/B of tools/librmr_base.so (tools/build_rev.sh REV tools/librmr_base.so) against the
# working tree's librmr.so on every hot kernel class: Cornell-5 (C2), RM3 builtin, the Mandelbulb (C3),
# csg256 (C4) and RM2 simple.scene, 1080p; bitwise comparison of the accumulators included.
#   SPP (default 16), ROUNDS (default 6), CASES (default: all five)
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
S=${SPP:-16}; R=${ROUNDS:-6}
run() {   # name, ab.py args
  local n=$1; shift
  timeout -k 10 240 python tools/ab.py tools/librmr_base.so raymarchrenderer_amd/librmr.so --rounds "$R" "$@" \
    > "gpurun_out/ab_$n.log" 2>&1 || return $?
  echo "== $n"; cat "gpurun_out/ab_$n.log"
}
C=" ${CASES:-c2 rm3 c3 c4 rm2} "   # subset, e.g. CASES="c4 c2"
[[ $C == *" c2 "* ]] && { run c2 --spp "$S" || exit $?; }
[[ $C == *" rm3 "* ]] && { run rm3 --scene builtin --variant 3 --bounces 16 --spp "$S" || exit $?; }
[[ $C == *" c3 "* ]] && { run c3 --scene scenes/mandelbulb.scene --bounces 2 --spp "$S" || exit $?; }
[[ $C == *" c4 "* ]] && { run c4 --scene scenes/csg256.scene --spp 8 || exit $?; }
[[ $C == *" rm2 "* ]] && { run rm2 --scene tests/golden/scenes/simple.scene --variant 2 --bounces 16 --spp "$S" || exit $?; }
exit 0
