#!/bin/bash
# Driver command (K = 20, W = 5) vs the untimed device warm-up length, interleaved on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abw
for rep in 1 2; do
  for w in ${WARMS:-200 500 1000 50}; do
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --device-warmup-ms $w > gpurun_out/abw/w${w}_$rep.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/abw/w${w}_$rep.log') if l.startswith('{')][-1]); print('warm $w rep $rep', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms_mean']*1e3,2))"
  done
done
