#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel-trace stats of the bench command, then PMC passes
# (counters only, one group per pass, no sys/runtime trace).  Summarise here with
#   python tools/profile_summary.py <round>     -> profiles/<round>_*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${1:-r01}
OUT=gpurun_out/$R
mkdir -p "$OUT/pmc"
export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:-"--no-cpu-baseline"}
echo "== bench (plain)"
timeout -k 10 300 python3 bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 bench.py $BENCH_ARGS > "$OUT/trace.log" 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "== pmc pass $i: $set"
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc/p$i" -o run -- \
    python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > "$OUT/pmc/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
