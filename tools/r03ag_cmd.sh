set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r03ag
CONFIGS="headline n16 n256" bash tools/pmc_configs.sh r03ag || exit $?
for c in headline n16 n256; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r03ag/prof_$c -o run -- python3 bench.py --config $c --steps 300 --no-cpu-baseline > gpurun_out/r03ag/prof_$c.log 2>&1 || exit $?
  echo "prof $c ok"
done
