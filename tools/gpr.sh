#!/bin/bash
# gpurun with waits for infrastructure transients only (exit 3 / "status=transient":
# nothing ran, nothing charged).  A command that ran and failed is never repeated.
# Usage: tools/gpr.sh <log> <timeout-s> '<command>'
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q -E "status=transient|backing off" "$LOG"; then sleep 75; continue; fi
  exit $rc
done
exit $rc
