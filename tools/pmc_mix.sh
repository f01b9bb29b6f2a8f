#!/bin/bash
# VALU instruction mix and VALU busy cycles of the headline step per build variant (diagnostic):
#   bash tools/pmc_mix.sh <tag> <variant>...   (build/var/<variant>.so; "prod" = the product library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:?tag}; shift
export TMPDIR=/tmp
for v in "$@"; do
  lib=build/var/$v.so; [ "$v" = prod ] && lib=""
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F64" \
             "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
             "SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"; do
    i=$((i+1)); d=gpurun_out/$T/pmc_$v/p$i; mkdir -p $d
    SWARM_MI355X_LIB=${lib:-} timeout -k 10 -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $d -o run -- python3 bench.py --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline > $d.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 $d.log; exit $rc; fi
  done
done
