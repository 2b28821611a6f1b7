#!/bin/bash
# Round-4 measurements in one GPU call (diagnostic library; logs in gpurun_out/r04ab_*.log):
# RM2's drain and section cycles, the C2 shading threshold, the certified getNormal probes on / off
# (C2's approximate map, C4's cache), RM2 wave targets, RM2's light-side shadow bound, C3's seeds in
# LDS, C4 without its sample-plane stores (timing bound).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 400 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -6
}
S=tests/golden/scenes/simple.scene
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ab_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04ab_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04ab_gpu_tests.log
export RMR_LIB=diag
run rm2_wave_times python -u tools/wave_times.py --variant rm2 --scene $S --bounces 16 --spp 4,16,64 || exit $?
RMR_JIT_OPTS=-DRMR_PROFILE run rm2_sections python -u tools/stats_run.py --variant rm2 --scene $S --bounces 16 --spp 4 || exit $?
run c2_cert python -u tools/env_ab.py RMR_JIT_CERT 1 0 --scenes cornell5 --rounds 5 --spp 16 || exit $?
run c4_cert python -u tools/env_ab.py RMR_JIT_OPTS "" "-DRMR_CACHE_CERT=0" --scenes csg256 --rounds 4 --spp 8 || exit $?
run rm2_waves python -u tools/env_ab.py RMR_JIT_OPTS "" "-DRMR_RM2_WAVES=6" "-DRMR_RM2_WAVES=8" --scenes rm2simple --rounds 4 --spp 16 || exit $?
run rm2_light python -u tools/env_ab.py RMR_JIT_OPTS "" "-DRMR_SHADOW_LIGHT_BOUND=0" --scenes rm2simple --rounds 6 --spp 16 || exit $?
run c3_seeds python -u tools/env_ab.py RMR_JIT_OPTS "" "-DRMR_SEED_LDS=0" --scenes mandelbulb --rounds 5 --spp 32 || exit $?
run c4_nostore python -u tools/env_ab.py RMR_JIT_OPTS "" "-DRMR_DIAG_NO_STORE" --scenes csg256 --rounds 4 --spp 8 || exit $?
run c2_shade_t python -u tools/env_ab.py shade_t 12 14 16 20 --scenes cornell5 --rounds 3 --spp 16 || exit $?
exit 0
