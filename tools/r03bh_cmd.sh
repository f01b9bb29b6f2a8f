#!/bin/bash
# Driver-length regions (rehearsed, events pre-created): eager 2 groups vs graph replay 2 / 4 groups.
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0 --region-reps 3"
for r in 1 2 3; do
  timeout -k 10 120 $B > gpurun_out/bh_eager_r${r}.txt 2>&1 || exit 1
  timeout -k 10 120 $B --graph-short > gpurun_out/bh_graph2_r${r}.txt 2>&1 || exit 1
  timeout -k 10 120 $B --graph-short --groups 4 > gpurun_out/bh_graph4_r${r}.txt 2>&1 || exit 1
done
