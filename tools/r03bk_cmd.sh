#!/bin/bash
# step64 with one select_topk call site (37.5 KB of code instead of 45.1 KB): parity, bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step64.py tests/test_gpu_parity.py tests/test_gpu_groups.py > gpurun_out/tk.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 180 python -u bench.py --no-cpu-baseline --cpu-variant-seconds 0 > gpurun_out/bk_def_r${r}.txt 2>&1 || exit 1
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0 --region-reps 3 > gpurun_out/bk_drv_r${r}.txt 2>&1 || exit 1
done
