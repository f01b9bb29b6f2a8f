set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/wu
for a in "--groups 2 --device-warmup-ms 0" "--groups 2 --device-warmup-ms 50" "--groups 2 --device-warmup-ms 200" "--groups 2 --device-warmup-ms 500" "--groups 1 --device-warmup-ms 200" "--groups 3 --device-warmup-ms 200" "--groups 2 --device-warmup-ms 200 --steps 500"; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $a > gpurun_out/wu/b.log 2>&1 || { tail -5 gpurun_out/wu/b.log; exit 3; }
  python -c "import json;d=json.loads(open('gpurun_out/wu/b.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$a', 'ms_per_step %.4f'%d['ms_per_step'], 'kern %.4f'%r['kernel_ms_mean'], 'eager %.4f'%d['ms_per_step_eager'], 'frac %.3f'%r['frac'], 'value %.3e'%d['value'], d['device_warmup'])"
done
