#!/bin/bash
# round 6: cache-served lanes join C4's full-map batches and re-anchor their cache (RMR_NPC_REFRESH)
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python tools/abrun.py --cases c4,csg64,csg_nodes --rounds 4 base="" refresh="opts:-DRMR_NPC_REFRESH=1" > $O/r06zj_npc_refresh.log 2>&1 || exit $?
timeout -k 10 600 python tools/abrun.py --cases c4 --rounds 2 pbase="opts:-DRMR_PROFILE" prefresh="opts:-DRMR_PROFILE -DRMR_NPC_REFRESH=1" >> $O/r06zj_npc_refresh.log 2>&1 || exit $?
grep '"case"' $O/r06zj_npc_refresh.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["case"], {k:(v["median_ms"],v["vs_first"],v["bitwise_equal_to_first"], v.get("sections"), v.get("lanes_per_full_batch")) for k,v in d.items() if isinstance(v,dict)})'
