#!/bin/bash
# Wait / memory attribution passes for one bench config (one counter group per rocprofv3 run,
# kernel trace only, as MI355X_MICROARCH.md's PMC section prescribes); summarise with
# tools/pmc_attr.py TAG.   tools/pmc_attr.sh TAG [CONFIG]   (CONFIG: bench.py --config, default c4)
cd "$(dirname "$0")/.." || exit 2
ROOTD=$(pwd); TAG=${1:-attr}; CFG=${2:-c4}
export TMPDIR=/tmp
B="$ROOTD/bench.py --config $CFG --overlap 0 --steps 1 --warmup 0 --no-cpu-baseline --no-psnr --no-count-pass"
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
PB="SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT"
PC="SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU"
PD="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
PE="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
PF="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITEBACK_sum TCC_NORMAL_EVICT_sum"
i=0
for P in "$PA" "$PB" "$PC" "$PD" "$PE" "$PF"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $P -d $ROOTD/gpurun_out/${TAG}_a$i -o run --output-format csv -- python3 $B > $ROOTD/gpurun_out/${TAG}_a$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
