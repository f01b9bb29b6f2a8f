set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
tail -3 gpurun_out/pt.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
bash tools/profile_round.sh r01
