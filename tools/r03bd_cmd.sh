#!/bin/bash
# Is the first K=20 region after the device warm-up slower than the following ones?
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0 --region-reps 8"
for r in 1 2; do
  for g in 2 4; do
    timeout -k 10 120 $B --groups $g > gpurun_out/bd_g${g}_r${r}.txt 2>&1 || exit 1
  done
done
