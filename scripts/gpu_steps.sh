#!/bin/bash
# Run GPU steps one after another, each under its own time limit. A step that fails
# its checks (exit 1, e.g. a pytest failure) does not stop the next one; a fault,
# abort, segfault or time-out (any other non-zero status) ends the script there.
# usage: scripts/gpu_steps.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: $name ended with status $rc"
    exit $rc
  fi
done
exit 0
