#!/bin/bash
# Runs GPU steps in order, each under its own time limit; stops at the first
# step that fails in any way (a failed test may be a GPU fault).
# usage: tools/gpu_steps.sh "SECONDS|NAME|COMMAND" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] $cmd (limit ${secs}s)"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc"
  tail -n 25 "gpurun_out/$name.log"
  # any failure ends the call: a failed test may be a GPU fault, and nothing
  # more may run on the GPU after one
  if [ $rc -ne 0 ]; then echo "=== stopping after [$name] (rc=$rc)"; exit $rc; fi
done
