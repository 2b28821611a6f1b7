#!/bin/bash
# round 6: candidate-grid cell records in 2x2x2 bricks (one 128-B line each) against the linear layout,
# then one PMC pass of L1->L2 request counts for each
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python tools/abrun.py --cases c4,csg64,csg_nodes --rounds 5 brick="" lin="env:RMR_GRID_BRICK=0" > $O/r06l_brick_ab.log 2>&1 || exit $?
grep '"case"' $O/r06l_brick_ab.log | cut -c1-3000
