#!/bin/bash
# Submit one gpurun call; when the pool has no box (nothing ran, nothing charged) wait and
# submit the same call again, at most 12 times.  Any call that ran is never repeated.
#   bash tools/gpurun_wait.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print(d.get('status'), d.get('run_s') or 0)" 2>/dev/null)
  case "$st" in
    "transient 0"*|"transient None"*) echo "[wait] no box (try $i), sleeping 240 s"; sleep 240 ;;
    *) exit $rc ;;
  esac
done
exit 3
