#!/bin/bash
# step16q speculative reset draws: parity with the variant library, then config-2 A/B.
set -o pipefail
mkdir -p gpurun_out/var
SWARM_MI355X_LIB=build/var/spec.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step16.py > gpurun_out/tu.txt 2>&1 || exit 1
for r in 1 2 3; do
  for v in base spec; do
    SWARM_MI355X_LIB=build/var/$v.so timeout -k 10 120 python bench.py --config n16 --no-cpu-baseline --cpu-variant-seconds 0 > gpurun_out/var/n16_${v}_$r.log 2>&1 || exit 1
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var/n16_${v}_$r.log)"
  done
done
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0 > gpurun_out/bu_drv.txt 2>&1 || exit 1
