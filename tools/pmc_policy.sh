#!/bin/bash
# PMC passes of the bf16 policy kernel in the rollout bench: bash tools/pmc_policy.sh <tag> [lib]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-ppmc}
export TMPDIR=/tmp
[ -n "${2:-}" ] && export SWARM_MI355X_LIB=$2
i=0
for set in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
  "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  d=gpurun_out/$T/p$i
  mkdir -p $d
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $d -o run -- python3 bench.py --policy bf16 --groups 1 --steps 20 --warmup 3 --device-warmup-ms 0 --no-cpu-baseline > $d.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -3 $d.log; exit $rc; }
done
