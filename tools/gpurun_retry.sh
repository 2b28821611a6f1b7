#!/bin/bash
# Run one gpurun call, retrying ONLY when the pool had no box for it (status "transient": nothing ran,
# nothing charged), with a pause between tries. Any other outcome (ok, fail, timeout) is final.
#   tools/gpurun_retry.sh TIMEOUT 'command'       (GPURUN_TRIES tries, default 8, GPURUN_WAIT s apart, default 90)
T=$1; shift
for i in $(seq 1 ${GPURUN_TRIES:-8}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c 'import json;print(json.load(open("gpurun_out/.last_call.json"))["status"])' 2>/dev/null)
  [ "$st" != transient ] && exit $rc
  echo "[gpurun_retry] no box (try $i), waiting ${GPURUN_WAIT:-90} s"
  sleep ${GPURUN_WAIT:-90}
done
exit $rc
