NB="--no-cpu-baseline --cpu-variant-seconds 0"
bash tools/gpu_steps.sh r05a \
 "suite:600:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "drv:150:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "launch2:200:SWARM_BENCH_REHEARSAL=1 python bench.py --gpus 2 --steps 20 --warmup 5 --envs 4096 $NB" \
 "gpus8:100:python bench.py --gpus 8 --steps 2 $NB; test \$? -ne 0" \
 "n16:120:python bench.py --config n16 --steps 200 --warmup 20 $NB" \
 "n256:120:python bench.py --config n256 --steps 200 --warmup 20 $NB" \
 "def:120:python bench.py $NB"
