#!/bin/bash
# Keyless pair pass for obstacle-collision / time-limit envs: parity, then bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step64.py tests/test_gpu_parity.py tests/test_gpu_groups.py tests/test_gpu_configs.py > gpurun_out/tg2.txt 2>&1 || exit 1
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0 --region-reps 4"
for r in 1 2 3; do
  timeout -k 10 120 $B > gpurun_out/bg_r${r}.txt 2>&1 || exit 1
done
timeout -k 10 180 python -u bench.py --no-cpu-baseline --cpu-variant-seconds 0 > gpurun_out/bg_def.txt 2>&1
