#!/bin/bash
# step64 straight-line general finish: parity tests, then A/B against the previous fallback.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step64.py tests/test_gpu_parity.py > gpurun_out/tl.txt 2>&1 || exit 1
VAR_BENCH_ARGS="--steps 400 --warmup 20" bash tools/run_variants.sh fb8 gen2 genfin fb8 gen2 genfin
