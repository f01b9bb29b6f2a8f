#!/bin/bash
# env-group sweep of the headline bench: bash tools/gpu_groups.sh "<G[:nograph]> ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/grp
export TMPDIR=/tmp
for spec in ${SPECS:-1 2 3 4 2:ng 3:ng 4:ng 1}; do
  G=${spec%%:*}; extra=""; [[ $spec == *:ng ]] && extra="--no-graph"
  timeout -k 10 120 python bench.py --groups $G $extra --no-cpu-baseline --steps 400 ${BENCH_ARGS:-} > gpurun_out/grp/b.log 2>&1 || { tail -5 gpurun_out/grp/b.log; exit 3; }
  python -c "import json;d=json.loads(open('gpurun_out/grp/b.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$spec', 'ms_per_step %.4f'%d['ms_per_step'], 'kern %.4f'%r['kernel_ms_mean'], 'eager %.4f'%d['ms_per_step_eager'], 'frac %.3f'%r['frac'], 'value %.3e'%d['value'])"
done
