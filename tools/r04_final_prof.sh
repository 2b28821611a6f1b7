#!/bin/bash
# Round-4 HEAD profiles of every bench config (tools/profile_round.sh: kernel-trace stats of the bench
# command, then the FETCH / WRITE / SQ / VALU PMC passes, each its own run), tags r04z_<config>.
# Then, on the build host: python tools/summarize_profile.py r04z_<config> <config> for each.
cd "$(dirname "$0")/.." || exit 2
for c in ${CONFIGS:-c2 c3 c4 c1 c5 rm2 rm3}; do
  st=3; [ $c = c4 ] && st=1; [ $c = c1 ] && st=50; [ $c = rm2 ] && st=20; [ $c = rm3 ] && st=10
  bash tools/profile_round.sh r04z_$c $c $st || exit $?
  echo "profiled $c"
done
