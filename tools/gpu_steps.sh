#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first fault / abort /
# timeout (exit >= 2 other than a plain test failure), as the pool rules require.
#   tools/gpu_steps.sh "<seconds>|<name>|<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] $cmd (limit ${secs}s)" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: step $name exited $rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
