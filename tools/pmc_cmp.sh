#!/bin/bash
# PMC instruction counts + kernel counters of one render per setting (tools/stats_run.py under rocprofv3
# --pmc; separate runs per setting). Usage: tools/pmc_cmp.sh TAG "ENV=.. ARGS" ["ENV=.. ARGS" ...]
#   e.g. tools/pmc_cmp.sh grid "RMR_GRID=1" "RMR_GRID=0"
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=(); args=()
  for w in $spec; do if [[ $w == *=* ]]; then envs+=("$w"); else args+=("$w"); fi; done
  env "${envs[@]}" timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmccmp_${TAG}_$i -o run --output-format csv -- python3 tools/stats_run.py "${args[@]}" > gpurun_out/pmccmp_${TAG}_$i.log 2>&1 || exit $?
  echo "== $spec"; grep '^{' gpurun_out/pmccmp_${TAG}_$i.log
done
