#!/bin/bash
# Diagnostic library variants that differ in ONE translation unit: recompile that unit with the
# given flags and link it with the product's other objects (build/obj, from __graft_entry__.build):
#   tools/variants_fast.sh name:unit:-DFLAG[,-DFLAG...] ...   ->  build/var/<name>.so
# unit: part0..part7 (swarm_kernel.hip SWARM_PART k), policy, eval
set -u
cd "$(dirname "$0")/.."
mkdir -p build/var/obj
CF="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -fno-slp-vectorize -mllvm -amdgpu-atomic-optimizer-strategy=None -I include"
C=multi-agent-rl-for-autonomous-drone-swarms_amd/csrc
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; unit=${rest%%:*}; flags=${rest#*:}; flags=${flags//,/ }
  case $unit in
    part*) src=$C/swarm_kernel.hip; defs="-DSWARM_PART=${unit#part}"; base=swarm_kernel.$unit.o
           # the product's per-part flags (__graft_entry__.PART_FLAGS): kernarg preload for parts 5, 6, 7
           case $unit in part5|part6|part7) defs="$defs -mllvm -amdgpu-kernarg-preload-count=16" ;; esac ;;
    policy) src=$C/swarm_policy.hip; defs=""; base=swarm_policy.o ;;
    eval) src=$C/swarm_eval.hip; defs=""; base=swarm_eval.o ;;
    *) echo "unknown unit $unit"; exit 2 ;;
  esac
  (hipcc $CF $defs $flags -c $src -o build/var/obj/$name.o 2>build/var/$name.err &&
   objs=$(ls build/obj/*.o | grep -v "/$base\$") &&
   hipcc --offload-arch=gfx950 -shared -fPIC $objs build/var/obj/$name.o -o build/var/$name.so 2>>build/var/$name.err) &
done
wait
ls -la build/var/*.so
