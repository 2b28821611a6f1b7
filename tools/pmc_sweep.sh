#!/bin/bash
# VALU/SALU instruction counts of the trace kernel per tuning setting (shade / refill thresholds):
# the slopes against the counters of tools/stats_run.py give the per-batch instruction costs.
export RMR_LIB=diag   # tools run against the diagnostic build (env switches)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for cfg in "16 2" "8 2" "32 2" "16 8" "16 16"; do
  set -- $cfg
  RMR_SHADE_T=$1 RMR_REFILL_T=$2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/sweep/s$1_r$2 -o run --output-format csv -- python3 tools/stats_run.py > gpurun_out/sweep/s$1_r$2.log 2>&1 || exit $?
done
echo sweep done
