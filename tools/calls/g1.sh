set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
tail -5 gpurun_out/pt.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for w in 4 5 6 8; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --waves-per-simd $w > gpurun_out/b_w$w.json 2> gpurun_out/b_w$w.err || exit 3
  python -c "import json;d=json.load(open('gpurun_out/b_w$w.json'));r=d['roofline'];print('wps',$w,'grid',r['grid'],'value %.3e'%d['value'],'kern_us %.1f'%(r['kernel_ms_mean']*1e3),'frac %.3f'%r['frac'])"
done
timeout -k 10 120 python bench.py --no-cpu-baseline --no-persistent > gpurun_out/b_np.json 2>/dev/null || exit 3
python -c "import json;d=json.load(open('gpurun_out/b_np.json'));r=d['roofline'];print('nonpersistent value %.3e'%d['value'],'kern_us %.1f'%(r['kernel_ms_mean']*1e3))"
