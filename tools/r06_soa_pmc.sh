#!/bin/bash
# round 6: LDS bank conflicts of the C4 cache kernel, AoS table (HEAD~ library) vs SoA (this tree), one
# counter group per rocprofv3 run (MI355X_MICROARCH.md), abrun's C4 case (1080p 8 spp), rows tile order
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out
mkdir -p /tmp/rp
for v in "aos=lib:tools/librmr_base.so" "soa=lib:raymarchrenderer_amd/librmr_diag.so"; do
  n=${v%%=*}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE -d /tmp/rp/$n -o run --output-format csv -- python3 tools/abrun.py --cases c4 --rounds 1 "$v" > $O/r06i_soa_pmc_$n.log 2>&1 || exit $?
  python3 tools/pmc_quick.py /tmp/rp/$n rmr_jit_trace $n | tee -a $O/r06i_soa_pmc.jsonl
done
