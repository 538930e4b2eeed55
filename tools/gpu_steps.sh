#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit; stop at the first step
# that faults, aborts, segfaults or times out (exit codes other than 0/1), so
# nothing else touches the GPU after trouble.
#   tools/gpu_steps.sh "<secs>|<name>|<command>" ...
# Output of each step goes to gpurun_out/<name>.log
set -u
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== step $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== step $name rc=$rc ($(( $(date +%s) - start ))s)"
  tail -n 5 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "=== stopping: step $name ended with rc=$rc"
    exit "$rc"
  fi
done
