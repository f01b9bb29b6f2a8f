bash tools/gpu_r03.sh r03bn \
 "t256:300:python -u -m pytest tests/test_gpu_step256.py tests/test_gpu_configs.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread" \
 "n256:200:python bench.py --config n256 --no-cpu-baseline --cpu-variant-seconds 0" \
 "n256b:200:python bench.py --config n256 --no-cpu-baseline --cpu-variant-seconds 0" \
 "def:200:python bench.py --no-cpu-baseline --cpu-variant-seconds 0"
