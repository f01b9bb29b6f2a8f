bash tools/gpu_r03.sh r03bw \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "drv:120:python bench.py --gpus 1 --steps 20 --warmup 5"
