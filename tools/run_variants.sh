#!/bin/bash
# On the GPU box: time each build/var/<name>.so with bench.py (and stamps for *stamps variants).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
export TMPDIR=/tmp
for name in "$@"; do
  so=build/var/$name.so
  if [[ $name == *stamps* ]]; then
    SWARM_STAMPS_DUMP=gpurun_out/var/$name.npz SWARM_STAMPS_LIB=$so timeout -k 10 120 python tools/stamps.py run > gpurun_out/var/$name.log 2>&1
  else
    SWARM_MI355X_LIB=$so timeout -k 10 120 python bench.py ${VAR_BENCH_ARGS:---steps 200 --warmup 20} --no-cpu-baseline --cpu-variant-seconds 0 > gpurun_out/var/$name.log 2>&1
  fi
  rc=$?
  echo "== $name rc=$rc $(grep -o "\"kernel_ms_mean\": [0-9.]*" gpurun_out/var/$name.log) $(grep -o "\"ms_per_step\": [0-9.]*" gpurun_out/var/$name.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 gpurun_out/var/$name.log; exit $rc; fi
done
