#!/bin/bash
# round 6: C4 cache kernel with 32-unit work chunks (4 KiB of LDS freed for a block-level full-map pool)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python tools/abrun.py --cases c4,csg64 --rounds 3 c64="" c32="opts:-DRMR_CHUNK_CACHE=32" > $O/r06f_c4_chunk32_ab.log 2>&1 || exit $?
grep '"case"' $O/r06f_c4_chunk32_ab.log | cut -c1-900
B="bench.py --config c4 --overlap 0 --steps 1 --warmup 0 --no-cpu-baseline --no-psnr --no-count-pass"
mkdir -p /tmp/rp
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT -d /tmp/rp/a2 -o run --output-format csv -- python3 $B > $O/r06f_c4lds_a2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d /tmp/rp/a1 -o run --output-format csv -- python3 $B > $O/r06f_c4lds_a1.log 2>&1 || exit $?
du -sh /tmp/rp/* ; find /tmp/rp -type f | head -20
for d in a1 a2; do mkdir -p $O/r06f_c4lds_$d; cp /tmp/rp/$d/*counter_collection.csv /tmp/rp/$d/*kernel_trace.csv $O/r06f_c4lds_$d/ 2>/dev/null; done
du -sh $O
echo done
