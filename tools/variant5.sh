#!/bin/bash
# Fast A/B variants of one kernel translation unit (PART=5: step64, the default; 6: step16q;
# 7: step256), linked with the other objects of the last build():
#   [PART=n] tools/variant5.sh name:-DFLAG[,-DFLAG...] ...  -> build/var/<name>.so
set -u
cd "$(dirname "$0")/.."
mkdir -p build/var
PART=${PART:-5}
others=$(ls build/obj/*.o | grep -v part$PART)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; flags=${flags//,/ }
  [ "$flags" = "$spec" ] && flags=""
  ( hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -I include -fno-slp-vectorize \
      -mllvm -amdgpu-atomic-optimizer-strategy=None -DSWARM_PART=$PART $flags -c \
      multi-agent-rl-for-autonomous-drone-swarms_amd/csrc/swarm_kernel.hip -o build/var/part5_$name.o 2>build/var/$name.err &&
    hipcc --offload-arch=gfx950 -shared -fPIC build/var/part5_$name.o $others -o build/var/$name.so ) &
done
wait
rm -f build/var/part5_*.o
ls -la build/var/*.so
