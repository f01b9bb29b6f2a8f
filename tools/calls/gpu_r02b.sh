#!/bin/bash
# GPU pass: full test suite, default bench, the driver's K/W, rocprofv3 stats of the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r02b}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$T/$name.log" 2>&1
  local rc=$?
  tail -n 3 "gpurun_out/$T/$name.log" | cut -c1-400
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
step bench 300 python bench.py
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python3 bench.py --steps 500 --no-cpu-baseline
