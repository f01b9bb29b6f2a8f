set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for e in 2048 4096 8192 16384 32768 65536; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-persistent --envs $e --steps 200 > gpurun_out/s_e$e.json 2>/dev/null || exit 3
  python -c "import json;d=json.load(open('gpurun_out/s_e$e.json'));r=d['roofline'];print('E',$e,'value %.3e'%d['value'],'kern_us %.1f'%(r['kernel_ms_mean']*1e3),'ns/env %.2f'%(r['kernel_ms_mean']*1e6/$e))"
done
