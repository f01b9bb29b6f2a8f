NB="--no-cpu-baseline --cpu-variant-seconds 0"
bash tools/gpu_steps.sh r04zh \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "drv:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "n16ev:200:python bench.py --config n16 --eval --steps 200 --warmup 20 $NB" \
 "evon:200:python bench.py --eval --steps 500 --warmup 50 $NB"
