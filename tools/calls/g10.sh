set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for a in "" "--no-term" ""; do
timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline $a > gpurun_out/nt.json 2>gpurun_out/nt.err || { tail -3 gpurun_out/nt.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/nt.json'));r=d['roofline'];print('$a','kern_us %.1f'%(r['kernel_ms_mean']*1e3),'value %.3e'%d['value'])"
done
