#!/bin/bash
# Multi-rank bench rehearsal on a one-GPU box: plain `bench.py --gpus N` launches N ranks itself;
# SWARM_BENCH_REHEARSAL=1 puts them all on cuda:0 over gloo.  bash tools/gpu_rehearsal.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-rehearsal}
mkdir -p gpurun_out/$T
export SWARM_BENCH_REHEARSAL=1
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --envs 4096 > gpurun_out/$T/r2.log 2>&1 || { tail -20 gpurun_out/$T/r2.log; exit 1; }
grep '^{' gpurun_out/$T/r2.log | cut -c1-300
timeout -k 10 300 python bench.py --gpus 4 --steps 20 --warmup 5 --envs 2048 > gpurun_out/$T/r4.log 2>&1 || { tail -20 gpurun_out/$T/r4.log; exit 1; }
grep '^{' gpurun_out/$T/r4.log | cut -c1-300
