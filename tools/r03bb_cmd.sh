#!/bin/bash
# swarm_step_groups: group tests, then driver-length bench lines with 2 / 4 env groups (alternating).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_groups.py > gpurun_out/tg.txt 2>&1 || exit 1
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0"
for r in 1 2 3; do
  for g in 2 4; do
    timeout -k 10 120 $B --groups $g > gpurun_out/bb_g${g}_r${r}.txt 2>&1 || exit 1
  done
done
timeout -k 10 120 $B > gpurun_out/bb_default.txt 2>&1
