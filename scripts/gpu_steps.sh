#!/bin/bash
# Runs GPU steps in order; each step has its own time limit. Stops at the first step that
# faulted / aborted / timed out (exit 124, 134, 137, 139 or >128) — test failures (exit 1) continue.
# usage: scripts/gpu_steps.sh "<name>:<seconds>:<command>" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  name="${step%%:*}"; rest="${step#*:}"
  secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] ($secs s) $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping after [$name] (rc=$rc)" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
