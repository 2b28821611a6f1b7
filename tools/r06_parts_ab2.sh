#!/bin/bash
# round 6: work-queue partitions 16 (kept) / 32 at every bench config's own spp
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python tools/abrun.py --cases rm3,rm2,c1,c2,c3,c4 --rounds 5 p16="" p32="opts:-DRMR_QUEUE_PARTS=32" > $O/r06z4_parts_ab2.log 2>&1 || exit $?
grep '"case"' $O/r06z4_parts_ab2.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["case"], d["spp"], {k:(v["median_ms"],v["vs_first"],v["bitwise_equal_to_first"]) for k,v in d.items() if isinstance(v,dict)})'
