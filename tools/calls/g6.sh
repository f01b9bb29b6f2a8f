set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
tail -15 gpurun_out/pt.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/b.json 2>gpurun_out/b.err || exit 3
python -c "import json;d=json.load(open('gpurun_out/b.json'));r=d['roofline'];print('value %.3e'%d['value'],'kern_us %.1f'%(r['kernel_ms_mean']*1e3),'frac %.3f'%r['frac'],r['kernel'])"
