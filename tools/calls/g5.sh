set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SWARM_STAMPS_DUMP=gpurun_out/stamps_once.npz timeout -k 10 120 python tools/stamps.py run > gpurun_out/stamps_once.txt 2>&1; rc=$?
cat gpurun_out/stamps_once.txt | grep -v amdgpu.ids; exit $rc
