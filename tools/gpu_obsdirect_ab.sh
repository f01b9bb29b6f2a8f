#!/bin/bash
# obs_direct A/B (SWARM_OBS_DIRECT=0/1) for small-N launches at three sizes, then the parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/od2
for e in 1024 8192 32768; do
  for od in 0 1; do
    SWARM_OBS_DIRECT=$od timeout -k 10 200 python3 bench.py --drones 16 --envs $e --groups 1 --no-cpu-baseline > gpurun_out/od2/e${e}_$od.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/od2/e${e}_$od.log') if l.startswith('{')][-1]); print('E=$e direct=$od', round(d['value']/1e9,3), round(d['ms_per_step']*1e3,2))"
  done
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread 2>&1 | tail -1
