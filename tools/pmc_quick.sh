#!/bin/bash
# Two SQ counter passes (instruction mix, issue/wait) of one bench config:
#   bash tools/pmc_quick.sh <tag> [config] [extra bench flags, e.g. "--dynamics physics"]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-q}; C=${2:-headline}; X=${3:-}
export TMPDIR=/tmp
i=0
for set in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  d=gpurun_out/$T/pmc_$C/p$i
  mkdir -p $d
  echo "== $C pass $i"
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $d -o run -- python3 bench.py --config $C --groups 1 --device-warmup-ms 0 --steps 40 --warmup 5 --no-cpu-baseline $X > $d.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 $d.log; echo "STOP (rc=$rc)"; exit $rc; fi
done
