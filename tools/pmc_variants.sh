#!/bin/bash
# PMC of diagnostic library variants (tools/variants_fast.sh -> build/var/<name>.so) on the headline
# shape, one counter pass per variant:  bash tools/pmc_variants.sh <tag> <name> ...
#   -> gpurun_out/<tag>/pmc_<name>/
# COUNTERS overrides the default set (LDS bank conflicts + issue counts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:?tag}; shift
export TMPDIR=/tmp
SET=${COUNTERS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"}
for name in "$@"; do
  d=gpurun_out/$T/pmc_$name/p1
  mkdir -p $d
  so=build/var/$name.so
  [ "$name" = base_lib ] && so=multi-agent-rl-for-autonomous-drone-swarms_amd/swarm_marl_amd/_lib/libswarm_mi355x.so
  echo "== $name"
  SWARM_MI355X_LIB=$so timeout -k 10 -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $d -o run -- python3 bench.py ${PMC_BENCH_ARGS:---groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline --cpu-variant-seconds 0} > $d.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -n 5 $d.log; echo "STOP (rc=$rc)"; exit $rc; fi
done
