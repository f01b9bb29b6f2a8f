#!/bin/bash
# Build ablation variants of the kernel library (here) or time them (on the GPU box: "run").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARIANTS="0 1 2 4 8 16 3 31"
if [ "${1:-build}" = build ]; then
  mkdir -p build/ablate
  for v in $VARIANTS; do
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -I include -DSWARM_ABLATE=$v \
      multi-agent-rl-for-autonomous-drone-swarms_amd/csrc/swarm_kernel.hip -o build/ablate/libswarm_abl$v.so &
  done
  wait
  ls -la build/ablate
else
  mkdir -p gpurun_out
  for v in $VARIANTS; do
    SWARM_MI355X_LIB=build/ablate/libswarm_abl$v.so timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/abl$v.log 2>&1
    rc=$?
    echo "variant $v rc=$rc $(grep -o '"kernel_ms_mean": [0-9.]*' gpurun_out/abl$v.log)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
fi
