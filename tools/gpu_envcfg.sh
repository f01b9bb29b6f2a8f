#!/bin/bash
# Per-env parameter tests first, then the whole GPU suite and the config lines.
# bash tools/gpu_envcfg.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-envcfg}
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
step envcfg 300 python -u -m pytest tests/test_gpu_env_cfg.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
step bench 300 python bench.py
step n16 300 python bench.py --config n16
step n256 300 python bench.py --config n256
