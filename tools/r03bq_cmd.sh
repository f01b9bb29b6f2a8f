#!/bin/bash
# Multi-rank rehearsal of the current bench (free bracket, rehearsals, native group launch):
# 2 and 4 ranks on cuda:0 over gloo, then a 2-rank CTDE gather run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_rehearsal.sh r03bq || exit 1
export SWARM_BENCH_REHEARSAL=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29515 bench.py --gpus 2 --steps 40 --warmup 5 --ctde --no-cpu-baseline --cpu-variant-seconds 0 \
  > gpurun_out/r03bq/ctde2.log 2>&1 || { tail -20 gpurun_out/r03bq/ctde2.log; exit 1; }
grep '^{' gpurun_out/r03bq/ctde2.log | cut -c1-300
