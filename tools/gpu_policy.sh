#!/bin/bash
# Policy kernel: GPU tests, rollout bench lines (bf16, f32), rocprofv3 kernel stats of the bf16 rollout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pol
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/pol/$name.log" 2>&1
  local rc=$?
  tail -n 6 "gpurun_out/pol/$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_policy 300 python -u -m pytest tests/test_gpu_policy.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step bench_pol_bf16 300 python bench.py --policy bf16 --no-cpu-baseline --steps 200
step bench_pol_f32 300 python bench.py --policy f32 --no-cpu-baseline --steps 40 --warmup 5
step prof_pol 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pol/prof -o run --output-format csv -- python3 bench.py --policy bf16 --no-cpu-baseline --steps 100 --warmup 10
