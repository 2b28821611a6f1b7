#!/bin/bash
# Round-4 HEAD: section cycles (RMR_PROFILE) of C2 / C3 / RM3 and the tail (tools/wave_times.py) of
# C2 / C3 / RM3 / C4 (diagnostic library); logs in gpurun_out/r04s_*.log.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export RMR_LIB=diag
run() {   # name, command...
  local n=$1; shift
  timeout -k 10 300 "$@" > "gpurun_out/r04s_$n.log" 2>&1 || return $?
  echo "== $n"; grep -v "amdgpu.ids" "gpurun_out/r04s_$n.log" | tail -4
}
RMR_JIT_OPTS=-DRMR_PROFILE run sec_c2 python -u tools/stats_run.py --spp 16 || exit $?
RMR_JIT_OPTS=-DRMR_PROFILE run sec_c3 python -u tools/stats_run.py --spp 16 --scene scenes/mandelbulb.scene --bounces 2 || exit $?
RMR_JIT_OPTS=-DRMR_PROFILE run sec_rm3 python -u tools/stats_run.py --spp 4 --scene builtin --variant rm3 --bounces 16 || exit $?
run wt_c2 python -u tools/wave_times.py --spp 16,64 || exit $?
run wt_rm3 python -u tools/wave_times.py --variant rm3 --scene builtin --bounces 16 --spp 4 || exit $?
run wt_rm2 python -u tools/wave_times.py --variant rm2 --scene tests/golden/scenes/simple.scene --bounces 16 --spp 4,16 || exit $?
exit 0
