#!/bin/bash
# Round-end check: full GPU suite, smoke(), default bench, rocprofv3 kernel stats of the default
# bench (and its trace for the union step time).  bash tools/gpu_final.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-final}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$T/$name.log" 2>&1
  local rc=$?
  tail -n 2 "gpurun_out/$T/$name.log" | cut -c1-250
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python3 bench.py
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python3 bench.py --steps 500 --no-cpu-baseline
