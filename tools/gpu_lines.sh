#!/bin/bash
# Bench lines of every measured variant (driver command included), one file each.
# bash tools/gpu_lines.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-lines}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$T/$name.log" 2>&1
  local rc=$?
  grep '^{' "gpurun_out/$T/$name.log" | tail -n 1 | cut -c1-160
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step headline 300 python3 bench.py
step noterm 300 python3 bench.py --no-term --cpu-seconds 2
step physics 300 python3 bench.py --dynamics physics --cpu-seconds 2
step n16 300 python3 bench.py --config n16 --cpu-seconds 2
step n256 300 python3 bench.py --config n256 --cpu-seconds 2
step rollout 300 python3 bench.py --policy bf16 --cpu-seconds 2
