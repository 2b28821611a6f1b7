#!/bin/bash
# round 6: work-queue partitions 16 (kept) / 32 / 64 — RM2 spends 54% of its wave cycles in claims
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/abrun.py --cases rm2,rm3,c1,c2 --spp 4 --rounds 5 p16="" p32="opts:-DRMR_QUEUE_PARTS=32" p64="opts:-DRMR_QUEUE_PARTS=64" > $O/r06z2_parts_ab.log 2>&1 || exit $?
grep '"case"' $O/r06z2_parts_ab.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["case"], {k:(v["median_ms"],v["vs_first"],v["bitwise_equal_to_first"]) for k,v in d.items() if isinstance(v,dict)})'
