#!/bin/bash
# Round-4 A/B, second part (diagnostic library; logs in gpurun_out/r04ab_*.log): certified probes of
# the cache kernels, RM2 wave targets, RM2's light-side shadow bound, C3's RNG state in LDS, C4
# without its sample-plane stores (timing bound), chunks per work-queue atomic (RMR_SUPER: a diagnostic
# option removed again once the partitioned queue replaced it), C2 shading threshold.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 400 "$@" > "gpurun_out/r04ab_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04ab_$n.log" | tail -6
}
E="python -u tools/env_ab.py"
run super $E --scenes rm2simple,rm3,cornell5 --rounds 4 --spp 16 RMR_JIT_OPTS -- "" "-DRMR_SUPER=2" "-DRMR_SUPER=4" "-DRMR_SUPER=8" || exit $?
RMR_JIT_OPTS="-DRMR_PROFILE -DRMR_SUPER=4" run rm2_sections_super4 python -u tools/stats_run.py --variant rm2 --scene tests/golden/scenes/simple.scene --bounces 16 --spp 4 || exit $?
run rm2_light $E --scenes rm2simple --rounds 6 --spp 16 RMR_JIT_OPTS -- "" "-DRMR_SHADOW_LIGHT_BOUND=0" || exit $?
run rm2_waves $E --scenes rm2simple --rounds 4 --spp 16 RMR_JIT_OPTS -- "" "-DRMR_RM2_WAVES=5" "-DRMR_RM2_WAVES=8" || exit $?
run c3_seeds $E --scenes mandelbulb --rounds 5 --spp 32 RMR_JIT_OPTS -- "" "-DRMR_SEED_LDS=0" || exit $?
run c4_cert $E --scenes csg256 --rounds 4 --spp 8 RMR_JIT_OPTS -- "" "-DRMR_CACHE_CERT=0" || exit $?
run c4_nostore $E --scenes csg256 --rounds 4 --spp 8 RMR_JIT_OPTS -- "" "-DRMR_DIAG_NO_STORE" || exit $?
run c4_super $E --scenes csg256 --rounds 3 --spp 8 RMR_JIT_OPTS -- "" "-DRMR_SUPER=4" || exit $?
run c2_shade_t $E --scenes cornell5 --rounds 3 --spp 16 shade_t -- 12 14 16 20 || exit $?
exit 0
