#!/bin/bash
# Round profile: kernel-trace stats of the bench command + PMC HBM-traffic passes (separate runs).
cd "$(dirname "$0")/.." || exit 2
ROOTD=$(pwd); TAG=${1:-r01}
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $ROOTD/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-psnr > $ROOTD/gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $ROOTD/gpurun_out/pmcf_$TAG -o run --output-format csv -- python3 $ROOTD/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-psnr > $ROOTD/gpurun_out/pmcf_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $ROOTD/gpurun_out/pmcw_$TAG -o run --output-format csv -- python3 $ROOTD/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-psnr > $ROOTD/gpurun_out/pmcw_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $ROOTD/gpurun_out/pmcs_$TAG -o run --output-format csv -- python3 $ROOTD/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-psnr > $ROOTD/gpurun_out/pmcs_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_FLAT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $ROOTD/gpurun_out/pmcv_$TAG -o run --output-format csv -- python3 $ROOTD/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-psnr > $ROOTD/gpurun_out/pmcv_$TAG.log 2>&1 || exit $?
echo profile done
