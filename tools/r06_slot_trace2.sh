#!/bin/bash
# round 6: full kernel timelines of the batched drop-in loop (RM3) with and without launch slots
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for ls in 0 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/slot_ls$ls -o run --output-format csv -- python3 bench.py --api render --config rm3 --steps 4 --warmup 1 --call-batching -1 --launch-streams $ls > $O/r06s_rm3_ls$ls.log 2>&1 || exit $?
  python3 tools/r06_timeline.py $ls || exit $?
done
wc -l $O/r06s_timeline_full_ls*.txt
