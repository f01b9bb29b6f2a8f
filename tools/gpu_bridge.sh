#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bridge
timeout -k 10 300 python -u -m pytest tests/test_gpu_bridge.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/bridge/pytest.log 2>&1; rc=$?; tail -25 gpurun_out/bridge/pytest.log; exit $rc
