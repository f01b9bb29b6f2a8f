#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dropin
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/dropin/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/dropin/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/dict_bench.py 3 3 4 16 64 > gpurun_out/dropin/dict.txt 2>&1; rc=$?; grep -v amdgpu gpurun_out/dropin/dict.txt; exit $rc
