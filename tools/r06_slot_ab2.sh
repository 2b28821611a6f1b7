#!/bin/bash
# round 6: adaptive launch slots (a slot only while the previous trace runs), one process per variant
# (no hardware-queue sharing between variants' streams): off, and slots with 0 / 32 / 64 reserved
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; mkdir -p $O
for v in off=0,0 r0=2,0 r32=2,32 r64=2,64; do
  timeout -k 10 300 python tools/slot_ab.py --cases rm3,c2,rm2 --spp 4 --rounds 5 $v > $O/r06u_slot_$v.log 2>&1 || exit $?
done
for f in $O/r06u_slot_*.log; do echo $f; grep '"case"' $f | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); k=[x for x in d if isinstance(d[x],dict)][0]; print(d["case"], d["pattern"], d[k]["median_ms"])'; done
