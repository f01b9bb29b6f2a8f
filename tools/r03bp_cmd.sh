#!/bin/bash
# kins_n (no inserts against empty slots): parity of the three specialisations, then A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step64.py tests/test_gpu_step16.py tests/test_gpu_step256.py tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/tp.txt 2>&1 || exit 1
VAR_BENCH_ARGS="--steps 400 --warmup 20" bash tools/run_variants.sh base new base new base new
