bash tools/gpu_r03.sh r03f \
 "suite:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "default:200:python bench.py --no-cpu-baseline" \
 "driver:200:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" \
 "noterm:200:python bench.py --no-term --no-cpu-baseline" \
 "var:300:bash tools/run_variants.sh a16"
