#!/bin/bash
# round 6: section cycles (RMR_PROFILE) of RM2 and RM3 at 1080p 4 spp
cd "$(dirname "$0")/.." || exit 2
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/abrun.py --cases rm2,rm3 --spp 4 --rounds 2 prof="opts:-DRMR_PROFILE" > $O/r06y_rm_sections.log 2>&1 || exit $?
grep '"case"' $O/r06y_rm_sections.log | cut -c1-1500
