#!/bin/bash
# Driver-length region: 2 vs 3 env groups in a fresh bench process each.
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0 --region-reps 3"
for r in 1 2 3; do
  for g in 2 3; do
    timeout -k 10 120 $B --groups $g > gpurun_out/br_g${g}_r${r}.txt 2>&1 || exit 1
  done
done
