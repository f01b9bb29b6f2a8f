#!/bin/bash
# Rehearsed driver-length regions: 4 runs of the driver's command with region reps.
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0 --region-reps 4"
for r in 1 2 3 4; do
  timeout -k 10 120 $B > gpurun_out/bf_r${r}.txt 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 120 $B --groups 4 > gpurun_out/bf_g4_r${r}.txt 2>&1 || exit 1
done
