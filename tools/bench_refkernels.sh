#!/bin/bash
# Bench lines + round profiles of the reference's own kernels (bench.py --config rm3 / rm2):
# RayMarch3.glsl as wired and the RM2 NEE variant, the configs whose CPU path (llvmpipe) was measured.
#   tools/bench_refkernels.sh TAG      logs: gpurun_out/bench_rm{3,2}.log, profiles via profile_round.sh
cd "$(dirname "$0")/.." || exit 2
TAG=${1:-r03a}
mkdir -p gpurun_out
for c in rm3 rm2; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 > gpurun_out/bench_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$c.log | cut -c1-400
done
for c in rm3 rm2; do
  bash tools/profile_round.sh ${TAG}_$c $c 5 || exit $?
done
