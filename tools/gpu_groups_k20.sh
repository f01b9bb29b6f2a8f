#!/bin/bash
# Driver-command timing (K = 20, W = 5) vs env groups, and K = 500 for reference, on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-gk20}
mkdir -p gpurun_out/$T
for rep in 1 2; do
  for g in 1 2 3; do
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --groups $g --no-cpu-baseline > gpurun_out/$T/k20_g${g}_$rep.log 2>&1 || { tail -5 gpurun_out/$T/k20_g${g}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$T/k20_g${g}_$rep.log') if l.startswith('{')][-1]); print('K20 g$g rep$rep', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_ms_mean']*1e3,1))"
  done
done
for g in 2 3; do
  timeout -k 10 200 python3 bench.py --groups $g --no-cpu-baseline > gpurun_out/$T/k500_g$g.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/$T/k500_g$g.log') if l.startswith('{')][-1]); print('K500 g$g', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,1))"
done
