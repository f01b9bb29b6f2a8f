set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
tail -3 gpurun_out/pt.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
b() { timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 --warmup 30 "$@" > gpurun_out/bx.json 2>gpurun_out/bx.err || { tail -3 gpurun_out/bx.err; exit 3; }
  python -c "import json,sys;d=json.load(open('gpurun_out/bx.json'));r=d['roofline'];print(sys.argv[1:],'kern_us %.1f'%(r['kernel_ms_mean']*1e3),'ms/step %.4f'%d['ms_per_step'],'value %.3e'%d['value'],r['kernel'])" "$@"; }
b
for w in 4 5 6; do b --waves-per-simd $w; done
b --envs 65536 --steps 100
for w in 6 8; do b --envs 65536 --steps 100 --waves-per-simd $w; done
b --envs 65536 --steps 100 --no-persistent
