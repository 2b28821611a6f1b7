#!/bin/bash
# round 6: C4 LDS table as SoA (A/B against the AoS HEAD library) + the LDS counters of the C4 launch;
# the C2 section split at HEAD (RMR_PROFILE)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python tools/abrun.py --cases c4,csg64 --rounds 3 base="lib:tools/librmr_base.so" soa="lib:raymarchrenderer_amd/librmr_diag.so" > $O/r06d_c4_soa_ab.log 2>&1 || exit $?
tail -4 $O/r06d_c4_soa_ab.log | cut -c1-600
timeout -k 10 300 python tools/abrun.py --cases c2 --spp 16 --rounds 2 prof="opts:-DRMR_PROFILE" > $O/r06d_c2_sections.log 2>&1 || exit $?
tail -2 $O/r06d_c2_sections.log | cut -c1-1500
B="bench.py --config c4 --overlap 0 --steps 1 --warmup 0 --no-cpu-baseline --no-psnr --no-count-pass"
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT -d $O/r06d_c4lds_a2 -o run --output-format csv -- python3 $B > $O/r06d_c4lds_a2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/r06d_c4lds_a1 -o run --output-format csv -- python3 $B > $O/r06d_c4lds_a1.log 2>&1 || exit $?
echo done
