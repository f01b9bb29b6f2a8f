#!/bin/bash
# Eval-metric kernel: parity tests, cost per step, rocprofv3 kernel stats.  bash tools/gpu_eval.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-eval}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$T/$name.log" 2>&1
  local rc=$?
  tail -n 3 "gpurun_out/$T/$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest tests/test_gpu_eval.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step bench64 200 python tools/eval_bench.py 8192 64 200
step bench16 200 python tools/eval_bench.py 1024 16 200
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run -- python tools/eval_bench.py 8192 64 100
