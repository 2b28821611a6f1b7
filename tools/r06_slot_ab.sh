#!/bin/bash
# round 6: launch slots against no slots, with 0 / 16 / 32 / 64 workgroups reserved for the folds
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python tools/slot_ab.py --cases rm3,c2,rm2 --spp 4 --rounds 5 off=0,0 r0=2,0 r16=2,16 r32=2,32 r64=2,64 > $O/r06t_slot_ab.log 2>&1 || exit $?
cat $O/r06t_slot_ab.log | cut -c1-1200
