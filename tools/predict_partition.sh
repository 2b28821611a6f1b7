#!/bin/bash
# One-GPU prediction of the N-rank tile partition (bench.py --predict) for C2, C4 and C5.
# Logs: gpurun_out/predict_<cfg>.log (last line = JSON)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c2 --predict 2,4,8 --steps 16 --warmup 2 > gpurun_out/predict_c2.log 2>&1 || exit $?
tail -1 gpurun_out/predict_c2.log | cut -c1-600
timeout -k 10 400 python bench.py --config c5 --predict 2,4,8 --steps 4 --warmup 1 > gpurun_out/predict_c5.log 2>&1 || exit $?
tail -1 gpurun_out/predict_c5.log | cut -c1-600
timeout -k 10 500 python bench.py --config c4 --predict 2,4,8 --steps 2 --warmup 1 > gpurun_out/predict_c4.log 2>&1 || exit $?
tail -1 gpurun_out/predict_c4.log | cut -c1-600
