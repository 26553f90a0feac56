#!/bin/bash
# Submit one gpurun call; when the pool has no box (nothing ran, nothing charged) wait as
# long as gpurun asks (its "retry in Ns", else 300 s) and submit the same call again, at
# most 12 times.  A call that ran is never repeated.
#   bash tools/gpurun_wait.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 1 12); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  echo "$out"
  st=$(python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print(d.get('status'), d.get('run_s') or 0)" 2>/dev/null)
  if echo "$out" | grep -q "status=transient" && { [ "$rc" = 3 ] || echo "$st" | grep -Eq "^transient (0|None)"; }; then
    w=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*" | tail -1)
    w=$(( ${w:-270} + 30 ))
    echo "[wait] no box (try $i), sleeping $w s"; sleep $w
  else
    exit $rc
  fi
done
exit 3
