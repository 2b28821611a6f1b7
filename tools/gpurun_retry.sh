#!/bin/bash
# Run one gpurun call, retrying ONLY when the pool had no box for it (status "transient": nothing ran,
# nothing charged), with a pause between tries. Any other outcome (ok, fail, timeout) is final.
#   tools/gpurun_retry.sh TIMEOUT 'command'       (at most 8 tries, 90 s apart)
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c 'import json;print(json.load(open("gpurun_out/.last_call.json"))["status"])' 2>/dev/null)
  [ "$st" != transient ] && exit $rc
  echo "[gpurun_retry] no box (try $i), waiting 90 s"
  sleep 90
done
exit $rc
