#!/bin/bash
# Round check: full GPU test suite, then the default bench line.  bash tools/gpu_check.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-chk}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$T/$name.log" 2>&1
  local rc=$?
  tail -n 4 "gpurun_out/$T/$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
step bench 300 python bench.py
