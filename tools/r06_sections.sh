#!/bin/bash
# round 6: section split (RMR_PROFILE) of C4 / csg64 / C3 at HEAD, lanes per full map() batch, and the
# LDS counters of the C4 launch with the SoA table
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python tools/abrun.py --cases c4,csg64,c3 --rounds 2 prof="opts:-DRMR_PROFILE" > $O/r06e_sections.log 2>&1 || exit $?
grep '"case"' $O/r06e_sections.log | cut -c1-900
B="bench.py --config c4 --overlap 0 --steps 1 --warmup 0 --no-cpu-baseline --no-psnr --no-count-pass"
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT -d $O/r06e_c4lds_a2 -o run --output-format csv -- python3 $B > $O/r06e_c4lds_a2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/r06e_c4lds_a1 -o run --output-format csv -- python3 $B > $O/r06e_c4lds_a1.log 2>&1 || exit $?
echo done
