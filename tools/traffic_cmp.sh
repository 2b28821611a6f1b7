#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate rocprofv3 passes) of one tools/stats_run.py render per
# setting. Usage: tools/traffic_cmp.sh TAG "ENV=.. ARGS" ["ENV=.. ARGS" ...]
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
  for ctr in FETCH_SIZE WRITE_SIZE; do
    env "${envs[@]}" timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/trf_${TAG}_${i}_$ctr -o run --output-format csv -- python3 tools/stats_run.py "${args[@]}" > gpurun_out/trf_${TAG}_${i}_$ctr.log 2>&1 || exit $?
  done
  python3 - "$spec" gpurun_out/trf_${TAG}_${i} <<'PY'
import csv, sys, collections
spec, base = sys.argv[1], sys.argv[2]
out = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    d = collections.defaultdict(float)
    for r in csv.DictReader(open("%s_%s/run_counter_collection.csv" % (base, ctr))):
        if "rmr_jit_trace" in r["Kernel_Name"] and r["Counter_Name"] == ctr:
            d[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    out[ctr] = d[max(d)] * 1024 / 1e9   # KiB -> GB, last launch
print(spec, {k: "%.2f GB" % v for k, v in out.items()})
PY
done
