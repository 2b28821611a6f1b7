#!/bin/bash
# Round profile: kernel-trace stats of the bench command + PMC passes (separate runs, one counter
# group each, as MI355X_MICROARCH.md's rocprofv3 section prescribes).
#   tools/profile_round.sh TAG [CONFIG] [STEPS]     (CONFIG = bench.py --config, default c2)
# Then (on the build host): python tools/summarize_profile.py TAG CONFIG
cd "$(dirname "$0")/.." || exit 2
ROOTD=$(pwd); TAG=${1:-r01}; CFG=${2:-c2}; STEPS=${3:-3}
export TMPDIR=/tmp
# --overlap 0 --launch-streams 0: one context without launch slots, so each launch runs alone (the bench
# line's roofline times launches the same way);
# tiles in row order unless TILE_ORDER=cost (C3: the cost probe's small launches would fill the traces)
B="$ROOTD/bench.py --config $CFG --overlap 0 --launch-streams 0 --tile-order ${TILE_ORDER:-rows} --no-cpu-baseline --no-psnr --no-count-pass"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $B --steps $STEPS --warmup 1 > $ROOTD/gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $ROOTD/gpurun_out/pmcf_$TAG -o run --output-format csv -- python3 $B --steps 1 --warmup 0 > $ROOTD/gpurun_out/pmcf_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $ROOTD/gpurun_out/pmcw_$TAG -o run --output-format csv -- python3 $B --steps 1 --warmup 0 > $ROOTD/gpurun_out/pmcw_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $ROOTD/gpurun_out/pmcs_$TAG -o run --output-format csv -- python3 $B --steps 1 --warmup 0 > $ROOTD/gpurun_out/pmcs_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_FLAT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $ROOTD/gpurun_out/pmcv_$TAG -o run --output-format csv -- python3 $B --steps 1 --warmup 0 > $ROOTD/gpurun_out/pmcv_$TAG.log 2>&1 || exit $?
echo profile done
