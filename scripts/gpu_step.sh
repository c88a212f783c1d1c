#!/usr/bin/env bash
# Run one GPU step under its own time limit; stop the whole session on a fault.
# usage: gpu_step.sh <seconds> <logname> <cmd...>
# exit codes 0/1 (test failures) continue; anything else (abort, segv, timeout) stops.
set -u
secs=$1; shift; log=$1; shift
mkdir -p gpurun_out
echo "[gpu_step] $(date +%T) start: $*" | tee -a gpurun_out/session.log
timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "[gpu_step] $(date +%T) rc=$rc: $*" | tee -a gpurun_out/session.log
tail -n 5 "gpurun_out/$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "[gpu_step] fatal rc=$rc -> stopping session" | tee -a gpurun_out/session.log
  exit 99
fi
exit 0
