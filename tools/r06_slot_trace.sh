#!/bin/bash
# round 6: kernel traces of the batched drop-in loop (RM3, one launch per frame) with and without launch
# slots, to see where a slotted frame loses time
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for ls in 0 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/slot_ls$ls -o run --output-format csv -- python3 bench.py --api render --config rm3 --steps 4 --warmup 1 --call-batching -1 --launch-streams $ls > $O/r06s_rm3_ls$ls.log 2>&1 || exit $?
  python3 tools/launch_gaps.py /tmp/slot_ls$ls/run_kernel_trace.csv --last 4 > $O/r06s_gaps_ls$ls.json || exit $?
  python3 - $ls <<'PY'
import csv, sys
ls = sys.argv[1]
rows = sorted(csv.DictReader(open("/tmp/slot_ls%s/run_kernel_trace.csv" % ls)), key=lambda r: int(r["Start_Timestamp"]))
t0 = None
out = open("gpurun_out/r06s_timeline_ls%s.txt" % ls, "w")
for r in rows[-40:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    t0 = t0 or s
    out.write("%10.1f %10.1f us  q%s grid %s  %s\n" % ((s - t0) / 1e3, (e - s) / 1e3, r["Queue_Id"], r["Grid_Size_X"], r["Kernel_Name"][:40]))
PY
done
tail -12 $O/r06s_timeline_ls0.txt; echo; tail -12 $O/r06s_timeline_ls2.txt
