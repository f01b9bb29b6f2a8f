#!/bin/bash
# Physics-mode checks: the GPU tests that cover it, then the physics bench line + kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-phys}
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
step tests 400 python -u -m pytest tests/test_gpu_step64.py tests/test_gpu_envs.py tests/test_gpu_parity.py tests/test_gpu_env_cfg.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step bench 300 python bench.py --dynamics physics
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python bench.py --dynamics physics --steps 300 --cpu-seconds 0.5
