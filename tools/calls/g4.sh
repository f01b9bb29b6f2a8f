set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/var; export TMPDIR=/tmp
b() { SWARM_MI355X_LIB=build/var/$1.so timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline ${@:2} > gpurun_out/var/$1.json 2>gpurun_out/var/$1.err || { tail -3 gpurun_out/var/$1.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/var/$1.json'));r=d['roofline'];print('$1 ${*:2}','kern_us %.1f'%(r['kernel_ms_mean']*1e3), 'value %.3e'%d['value'], 'grid', r['grid'])"; }
for v in "$@"; do b $v; done
