#!/bin/bash
# GPU round check: parity tests -> smoke -> bench -> rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault/abort/timeout (rc not in {0,1}) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 25 "gpurun_out/$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 480 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240
  step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 300 python bench.py
  step bench_noterm 300 python bench.py --no-term --no-cpu-baseline
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline
  find gpurun_out/prof -name "*stats*" | head
fi
