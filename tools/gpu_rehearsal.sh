#!/bin/bash
# Multi-rank bench rehearsal on a one-GPU box: 2 ranks on cuda:0 over gloo (torchrun), then the
# same for 4 ranks with 2048 envs each.  bash tools/gpu_rehearsal.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-rehearsal}
mkdir -p gpurun_out/$T
export SWARM_BENCH_REHEARSAL=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29513 bench.py --gpus 2 --steps 20 --warmup 5 --envs 4096 > gpurun_out/$T/r2.log 2>&1 || { tail -20 gpurun_out/$T/r2.log; exit 1; }
grep '^{' gpurun_out/$T/r2.log | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29514 bench.py --gpus 4 --steps 20 --warmup 5 --envs 2048 > gpurun_out/$T/r4.log 2>&1 || { tail -20 gpurun_out/$T/r4.log; exit 1; }
grep '^{' gpurun_out/$T/r4.log | cut -c1-300
