bash tools/gpu_r03.sh r03i \
 "suite:600:python -u -m pytest tests/test_gpu_step64.py tests/test_gpu_parity.py tests/test_gpu_groups.py -x -q --timeout 120 --timeout-method thread" \
 "default:200:python bench.py --no-cpu-baseline" \
 "default2:200:python bench.py --no-cpu-baseline" \
 "noterm:200:python bench.py --no-term --no-cpu-baseline"
