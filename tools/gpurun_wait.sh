#!/bin/bash
# Build-host helper: submit one gpurun command, re-submitting only while the pool reports
# "no box free" (exit 3: nothing ran, nothing charged).  Any other outcome ends the loop.
#   bash tools/gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  echo "[gpurun_wait] try $i: no box, retrying in 150 s" >> "$LOG.tries"
  sleep 150
done
echo "[gpurun_wait] rc=$rc" >> "$LOG"
exit $rc
