#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/physab
timeout -k 10 300 python -u -m pytest tests/test_gpu_step64.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k physics > gpurun_out/physab/tests.log 2>&1 || { tail -20 gpurun_out/physab/tests.log; exit 1; }
tail -1 gpurun_out/physab/tests.log
timeout -k 10 300 python bench.py --dynamics physics --cpu-seconds 0.5 > gpurun_out/physab/bench.log 2>&1 || exit 1
grep '^{' gpurun_out/physab/bench.log | cut -c1-300
bash tools/pmc_quick.sh physab headline "--dynamics physics"
