#!/bin/bash
# round profiles of C2, C3 and C4 (tools/profile_round.sh) with tag TAG
cd "$(dirname "$0")/.." || exit 2
TAG=${1:-r03}
bash tools/profile_round.sh $TAG c2 3 || exit $?
bash tools/profile_round.sh ${TAG}_c3 c3 3 || exit $?
bash tools/profile_round.sh ${TAG}_c4 c4 1 || exit $?
