#!/bin/bash
# usage: tools/gpu_try.sh LOG TIMEOUT 'command'   -- retries only when the pool has no free box / slot (nothing charged)
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "no free box right now\|GPU slot(s) on this pod are busy\|backing off after the last attempt failed on the infrastructure" "$LOG"; then
    sleep 150; continue
  fi
  exit $rc
done
exit 3
