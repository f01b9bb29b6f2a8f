#!/bin/bash
# step256 XOR mirror keys: parity tests, then config-5 slab lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step256.py tests/test_gpu_configs.py > gpurun_out/ti.txt 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 180 python -u bench.py --config n256 --no-cpu-baseline --cpu-variant-seconds 0 > gpurun_out/bi_n256_r${r}.txt 2>&1 || exit 1
done
