#!/bin/bash
# Round-2 evidence: the three config bench lines (with CPU baselines), rocprofv3 kernel stats of
# each, PMC passes of all three (tools/pmc_configs.sh).  bash tools/gpu_r02_final.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r02f}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$T/$name.log" 2>&1
  local rc=$?
  tail -n 1 "gpurun_out/$T/$name.log" | cut -c1-200
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
for c in headline n16 n256; do
  step bench_$c 300 python bench.py --config $c
  step prof_$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 500 --no-cpu-baseline
done
bash tools/pmc_configs.sh $T
