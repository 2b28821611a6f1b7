#!/bin/bash
# round 6: RM2 hands out all its work by 31% of the launch (r06z5_wave_times_rm2.log): smaller chunks
# (units per claim) for the non-cache kernels, 128 (kept) / 96 / 64
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python tools/abrun.py --cases rm2,rm3,c1,c2,c3 --spp 4 --rounds 5 k128="" k96="opts:-DRMR_CHUNK=96" k64="opts:-DRMR_CHUNK=64" > $O/r06z6_chunk_rm.log 2>&1 || exit $?
grep '"case"' $O/r06z6_chunk_rm.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["case"], d["spp"], {k:(v["median_ms"],v["vs_first"],v["bitwise_equal_to_first"]) for k,v in d.items() if isinstance(v,dict)})'
