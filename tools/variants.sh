#!/bin/bash
# Build diagnostic single-unit variants of the kernel library in parallel:
#   tools/variants.sh name:-DFLAG[,-DFLAG...] ...   ->  build/var/<name>.so
set -u
cd "$(dirname "$0")/.."
mkdir -p build/var
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; flags=${flags//,/ }
  [ "$flags" = "$spec" ] && flags=""
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -I include -fno-slp-vectorize -mllvm -amdgpu-atomic-optimizer-strategy=None $flags \
    multi-agent-rl-for-autonomous-drone-swarms_amd/csrc/swarm_kernel.hip multi-agent-rl-for-autonomous-drone-swarms_amd/csrc/swarm_policy.hip multi-agent-rl-for-autonomous-drone-swarms_amd/csrc/swarm_eval.hip -o build/var/$name.so 2>build/var/$name.err &
done
wait
ls -la build/var/*.so
