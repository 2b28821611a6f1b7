#!/bin/bash
# Round-end profiles of the given bench configs at HEAD: tools/profile_round.sh TAG_<cfg> <cfg> for each
# (rocprofv3 kernel stats + separate PMC passes), then summarise them into profiles/ on the build host
# (python tools/summarize_profile.py TAG_<cfg> <cfg>).   tools/round_profiles.sh TAG cfg [cfg ...]
cd "$(dirname "$0")/.." || exit 2
TAG=$1; shift
for c in "$@"; do
  st=3; [ $c = c1 ] && st=20; [ $c = rm3 ] && st=10; [ $c = rm2 ] && st=20; [ $c = c4 ] && st=2; [ $c = c5 ] && st=2
  bash tools/profile_round.sh ${TAG}_$c $c $st > gpurun_out/${TAG}_$c.log 2>&1 || { echo "profile $c failed"; exit 1; }
  echo "profile $c done"
done
