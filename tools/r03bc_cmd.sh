#!/bin/bash
# Free-bracket eager region: driver-length bench lines with 2 / 4 env groups (alternating).
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0"
for r in 1 2 3 4; do
  for g in 2 4; do
    timeout -k 10 120 $B --groups $g > gpurun_out/bc_g${g}_r${r}.txt 2>&1 || exit 1
  done
done
