#!/bin/bash
# PMC passes (counters only, --kernel-trace/--stats style: no sys/runtime trace) on a short bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 40 --warmup 5 --no-cpu-baseline"}
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for set in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU_FP64 SQ_INSTS_VALU_CVT SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -k 10 180 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 3 gpurun_out/pmc/p$i.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP (rc=$rc)"; exit $rc; fi
done
