#!/bin/bash
# Eval kernel ablations (build/var/eval_abl{1,2}.so): rocprofv3 kernel stats per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-evabl}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for v in 0 1 2 3 4 5; do
  if [ $v -eq 0 ]; then unset SWARM_MI355X_LIB; else export SWARM_MI355X_LIB=$PWD/build/var/eval_abl$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/v$v -o run -- python tools/eval_bench.py 8192 64 100 > gpurun_out/$T/v$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "variant $v ok"
done
