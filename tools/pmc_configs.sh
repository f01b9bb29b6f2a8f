#!/bin/bash
# PMC passes (counters only; no sys/runtime trace) for the three bench configs, one counter group
# per pass and per config:  bash tools/pmc_configs.sh [round]  ->  gpurun_out/<round>/pmc_<config>/p*/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${1:-r02}
export TMPDIR=/tmp
# PMC_SETS (optional): counter groups separated by ';' instead of the default four passes
if [ -n "${PMC_SETS:-}" ]; then IFS=';' read -r -a SETS <<< "$PMC_SETS"; else SETS=(
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
    "FETCH_SIZE" "WRITE_SIZE"); fi
for c in ${CONFIGS:-headline n16 n256}; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    d=gpurun_out/$R/pmc_$c/p$i
    mkdir -p $d
    echo "== $c pass $i: $set"
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $d -o run -- python3 bench.py --config $c --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline > $d.log 2>&1
    rc=$?
    echo "rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -n 5 $d.log; echo "STOP (rc=$rc)"; exit $rc; fi
  done
done
