#!/bin/bash
# Kernel time vs env count / drones (diagnostic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for args in "--envs 512" "--envs 1024" "--envs 2048" "--envs 4096" "--envs 8192" "--envs 16384" "--envs 32768" "--drones 32 --envs 16384" "--drones 16 --envs 32768" ${EXTRA:-}; do
  timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline $args > gpurun_out/sweep.log 2>&1
  rc=$?
  echo "$args rc=$rc $(grep -o '"kernel_ms_mean": [0-9.]*' gpurun_out/sweep.log) $(grep -o '"value": [0-9.e+]*' gpurun_out/sweep.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
