set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/var; export TMPDIR=/tmp
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/b.json'));r=d['roofline'];print('graph value %.3e'%d['value'],'ms/step %.4f eager %.4f'%(d['ms_per_step'],d['ms_per_step_eager']),'kern_us %.1f'%(r['kernel_ms_mean']*1e3))"
bash tools/g4.sh base noslp
