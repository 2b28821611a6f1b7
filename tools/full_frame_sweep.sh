#!/bin/bash
# Full-frame bitwise sweep of the exact work-skipping paths (rmr_set_culling all on vs all off) per
# scene family, at production sizes; differing samples are checked against the CPU oracle.
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
O=gpurun_out/full_frame_sweep.log; : > $O
run() { echo "== $*" >> $O; timeout -k 10 300 python tools/mode_diff.py culling 7 0 "$@" >> $O 2>&1 || exit $?; }
run --scene scenes/cornell5.scene --spp 4 --bounces 4
run --scene tests/golden/scenes/glass_test.scene --spp 2 --bounces 16
run --scene tests/golden/scenes/default.scene --spp 2 --bounces 16
run --scene tests/golden/scenes/multilight.scene --spp 2 --bounces 16
run --scene tests/golden/scenes/simple.scene --variant rm2 --spp 4 --bounces 16
run --scene builtin --variant rm3 --spp 4 --bounces 16
run --scene scenes/mandelbulb.scene --spp 2 --bounces 2
run --scene scenes/csg256.scene --spp 2 --bounces 4 --W 1920 --H 1080
run --scene scenes/csg64.scene --spp 2 --bounces 4
grep -v amdgpu.ids $O
