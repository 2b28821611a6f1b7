#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over a short bench run.
# usage: tools/pmc.sh <tag> [bench args...]
cd "$(dirname "$0")/.." || exit 2
ROOTD=$(pwd)
TAG=${1:-pmc}; shift
ARGS=${@:-"--spp 8 --steps 1 --warmup 0 --no-cpu-baseline"}
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_FLAT SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
P4="WRITE_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P -d $ROOTD/gpurun_out/${TAG}_p$i -o run --output-format csv -- python3 $ROOTD/bench.py $ARGS > $ROOTD/gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
