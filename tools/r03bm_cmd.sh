bash tools/gpu_r03.sh r03bm \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread" \
 "def:200:python bench.py --no-cpu-baseline --cpu-variant-seconds 0" \
 "drv:120:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0 --region-reps 3" \
 "drv2:120:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0 --region-reps 3" \
 "n256:200:python bench.py --config n256 --no-cpu-baseline --cpu-variant-seconds 0" \
 "n16:200:python bench.py --config n16 --no-cpu-baseline --cpu-variant-seconds 0"
