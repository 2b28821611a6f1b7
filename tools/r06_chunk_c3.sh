#!/bin/bash
# round 6: chunk size 128 (kept) / 96 / 64 for the Mandelbulb (C3) and Cornell-5 (C2) at 16 spp
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python tools/abrun.py --cases c3,c2 --rounds 5 k128="" k96="opts:-DRMR_CHUNK=96" k64="opts:-DRMR_CHUNK=64" > $O/r06z7_chunk_c3.log 2>&1 || exit $?
timeout -k 10 900 python tools/abrun.py --cases c3 --spp 64 --rounds 3 k128="" k64="opts:-DRMR_CHUNK=64" >> $O/r06z7_chunk_c3.log 2>&1 || exit $?
grep '"case"' $O/r06z7_chunk_c3.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["case"], d["spp"], {k:(v["median_ms"],v["vs_first"],v["bitwise_equal_to_first"]) for k,v in d.items() if isinstance(v,dict)})'
