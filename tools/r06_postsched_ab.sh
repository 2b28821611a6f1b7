#!/bin/bash
# round 6: the post-RA machine scheduler (fills VALU hazard wait states with independent instructions)
# on the inline-map kernels, against the kept max-memory-clause-without-post-RA choice
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python tools/abrun.py --cases c2,c3,rm3,c1 --rounds 4 pm0="" pm1="env:RMR_JIT_POSTSCHED=1" dflt="env:RMR_JIT_SCHED=0" > $O/r06k_postsched_ab.log 2>&1 || exit $?
grep '"case"' $O/r06k_postsched_ab.log | python3 -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['case'], {k:(v['median_ms'], v['vs_first'], v['bitwise_equal_to_first']) for k,v in d.items() if isinstance(v, dict)})"
