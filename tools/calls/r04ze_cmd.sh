NB="--no-cpu-baseline --cpu-variant-seconds 0"
bash tools/gpu_steps.sh r04ze \
 "drv1:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "evon:200:python bench.py --eval --steps 500 --warmup 50 $NB" \
 "evoff:200:python bench.py --no-graph --steps 500 --warmup 50 $NB" \
 "drv2:120:python bench.py --gpus 1 --steps 20 --warmup 5 $NB" \
 "evon2:200:python bench.py --eval --steps 500 --warmup 50 $NB" \
 "evoff2:200:python bench.py --no-graph --steps 500 --warmup 50 $NB" \
 "drv3:120:python bench.py --gpus 1 --steps 20 --warmup 5 $NB" \
 "def:300:python bench.py $NB" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread"
