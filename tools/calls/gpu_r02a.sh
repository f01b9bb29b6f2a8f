#!/bin/bash
# Round-2 GPU pass: full GPU test suite, the three config bench lines, rocprofv3 kernel stats of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/r02/$name.log" 2>&1
  local rc=$?
  tail -n 4 "gpurun_out/r02/$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
step bench_headline 300 python bench.py
step bench_n16 300 python bench.py --config n16
step bench_n256 300 python bench.py --config n256
for c in headline n16 n256; do
  step prof_$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 300 --warmup 20 --no-cpu-baseline
done
