#!/bin/bash
# step16q kins_n: parity, then config-2 A/B (alternating).
set -o pipefail
mkdir -p gpurun_out/var
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step16.py tests/test_gpu_configs.py > gpurun_out/tt.txt 2>&1 || exit 1
for r in 1 2 3; do
  for v in base new; do
    SWARM_MI355X_LIB=build/var/$v.so timeout -k 10 120 python bench.py --config n16 --no-cpu-baseline --cpu-variant-seconds 0 > gpurun_out/var/n16_${v}_$r.log 2>&1 || exit 1
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var/n16_${v}_$r.log)"
  done
done
