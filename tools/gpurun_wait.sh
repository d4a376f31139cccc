#!/bin/bash
# Submit one gpurun call; when the pool had no slot or box for it (status "transient": nothing ran, nothing was
# charged) wait a few minutes and submit it again, at most 20 times. Any call that ran — passed or failed — ends it.
#   usage: bash tools/gpurun_wait.sh <log> <timeout_s> '<command>'
LOG=$1; TMO=$2; CMD=$3
for i in $(seq 1 20); do
  timeout $((TMO + 900)) /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && ! grep -q "status=ok\|status=fail" "$LOG"; then
    echo "[wait] attempt $i: no slot / box ($(grep -o 'status=transient.*' "$LOG" | head -1 | cut -c1-80)); sleeping" >> "$LOG.wait"
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
