#!/bin/bash
# The reference's call pattern through the drop-in: bench.py --api render lines for
# C2 and RM3, the C++ host's per-sample loop (rmr_cli --per-sample) beside its batched one, and a
# rocprofv3 kernel trace of the per-call loop for the launch gaps (tools/launch_gaps.py).
#   tools/api_render_probe.sh TAG
cd "$(dirname "$0")/.." || exit 2
ROOTD=$(pwd); TAG=${1:-r06}
export TMPDIR=/tmp
O=$ROOTD/gpurun_out
for c in c2 rm3; do for cb in -1 0; do
  timeout -k 10 300 python3 bench.py --api render --config $c --steps 3 --warmup 1 --call-batching $cb > $O/api_${TAG}_${c}_cb$cb.log 2>&1 || exit $?
  tail -1 $O/api_${TAG}_${c}_cb$cb.log; done
done
CLI=$ROOTD/raymarchrenderer_amd/rmr_cli
for m in "--per-sample" ""; do
  timeout -k 10 300 $CLI --scene scenes/cornell5.scene --size 1920x1080 --samples 64 --bounces 4 --out /tmp/cli.bmp $m > $O/cli_${TAG}_c2${m}.log 2>&1 || exit $?
  grep msamples $O/cli_${TAG}_c2${m}.log
done
for cb in 0 -1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/apiprof_${TAG}_cb$cb -o run --output-format csv -- python3 bench.py --api render --config c2 --steps 1 --warmup 1 --spp 16 --call-batching $cb > $O/apiprof_${TAG}_cb$cb.log 2>&1 || exit $?
  python3 tools/launch_gaps.py $O/apiprof_${TAG}_cb$cb/run_kernel_trace.csv --last $([ $cb = 0 ] && echo 256 || echo 1) > $O/apigaps_${TAG}_cb$cb.json && cat $O/apigaps_${TAG}_cb$cb.json
done
