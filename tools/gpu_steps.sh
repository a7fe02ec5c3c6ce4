#!/bin/bash
# tools/gpu_steps.sh <log> <step>... -- run GPU steps in order, each under its own time limit
# (the step strings are "SECONDS command..."), stopping at the first step that fails with
# anything but an ordinary test failure (exit 1): a fault, an abort or a time limit ends the
# sequence, so nothing more runs on a GPU in a bad state.
LOG=$1; shift
for st in "$@"; do
  secs=${st%% *}; cmd=${st#* }
  echo "=== [$secs s] $cmd" >> "$LOG"
  timeout -k 10 "$secs" bash -c "$cmd" >> "$LOG" 2>&1
  rc=$?
  echo "=== rc=$rc" >> "$LOG"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
exit 0
