#!/bin/bash
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probes/sqrt_exhaustive > gpurun_out/sqrt_exh.log 2>&1; echo "sqrt rc=$?"; cat gpurun_out/sqrt_exh.log
timeout -k 10 300 python tools/tune.py --spp 16 --configs "$(cat tools/tune_cf.json)" > gpurun_out/tune_r1d.log 2>&1 || exit $?
cat gpurun_out/tune_r1d.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['cfg'], d['Msamples/s'], d['trace_ms'], d['lane_util'])"
