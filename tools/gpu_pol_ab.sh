#!/bin/bash
# Policy A/B: the in-tree library vs build/var/pol_<variant>.so (tools/policy_scale.py), then the
# policy parity tests on the in-tree one.  bash tools/gpu_pol_ab.sh <tag> <variant...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-polab}; shift
mkdir -p gpurun_out/$T
timeout -k 10 200 python tools/policy_scale.py > gpurun_out/$T/cur.log 2>&1 || { tail -5 gpurun_out/$T/cur.log; exit 1; }
echo "cur $(tail -1 gpurun_out/$T/cur.log)"
for v in "$@"; do
  SWARM_MI355X_LIB=$PWD/build/var/pol_$v.so timeout -k 10 200 python tools/policy_scale.py > gpurun_out/$T/$v.log 2>&1 || { tail -5 gpurun_out/$T/$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/$T/$v.log)"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -1 gpurun_out/$T/tests.log
exit $rc
