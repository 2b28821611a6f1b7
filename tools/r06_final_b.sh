#!/bin/bash
# round-6 measurement set, part B: rocprofv3 kernel stats + PMC passes per config (round_profiles.sh),
# then the one-GPU N-rank partition prediction (predict_partition.sh)
cd "$(dirname "$0")/.." || exit 2
TAG=${1:-r06y}
mkdir -p gpurun_out
bash tools/round_profiles.sh $TAG c1 c2 c3 c4 c5 rm2 rm3 || exit $?
bash tools/predict_partition.sh || exit $?
