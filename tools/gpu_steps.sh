#!/bin/bash
# GPU step runner: bash tools/gpu_steps.sh <tag> <name>:<timeout>:<command> ...
# Every step runs under its own timeout; the first failing step ends the call (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:?tag}; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; to=${rest%%:*}; cmd=${rest#*:}
  echo "== $name"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$T/$name.log" 2>&1
  rc=$?
  grep -E '^\{|passed|failed|error' "gpurun_out/$T/$name.log" | tail -n 2 | cut -c1-600
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 15 "gpurun_out/$T/$name.log"; echo "STOP after $name (rc=$rc)"; exit $rc; fi
done
