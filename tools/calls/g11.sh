set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for e in 2048 4096 8192 16384 32768 65536; do
timeout -k 10 120 python bench.py --envs $e --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/es.json 2>gpurun_out/es.err || { tail -3 gpurun_out/es.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/es.json'));r=d['roofline'];k=r['kernel_ms_mean']*1e3;print('E=$e','kern_us %.1f'%k,'ns/env %.2f'%(k*1e3/$e),'value %.3e'%d['value'],'frac %.3f'%r['frac'])"
done
