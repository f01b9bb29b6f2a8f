#!/bin/bash
# Fast A/B variants of the step64 translation unit (SWARM_PART=5) only, linked with the other
# objects of the last build():  tools/variant5.sh name:-DFLAG[,-DFLAG...] ...  -> build/var/<name>.so
set -u
cd "$(dirname "$0")/.."
mkdir -p build/var
others=$(ls build/obj/*.o | grep -v part5)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; flags=${flags//,/ }
  [ "$flags" = "$spec" ] && flags=""
  ( hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -I include -fno-slp-vectorize \
      -mllvm -amdgpu-atomic-optimizer-strategy=None -DSWARM_PART=5 $flags -c \
      multi-agent-rl-for-autonomous-drone-swarms_amd/csrc/swarm_kernel.hip -o build/var/part5_$name.o 2>build/var/$name.err &&
    hipcc --offload-arch=gfx950 -shared -fPIC build/var/part5_$name.o $others -o build/var/$name.so ) &
done
wait
rm -f build/var/part5_*.o
ls -la build/var/*.so
