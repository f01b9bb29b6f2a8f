bash tools/gpu_r03.sh r03o \
 "step16:400:python -u -m pytest tests/test_gpu_step16.py -x -q --timeout 120 --timeout-method thread" \
 "parity:400:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_envs.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread" \
 "n16:150:python bench.py --config n16 --no-cpu-baseline" \
 "n16b:150:python bench.py --config n16 --no-cpu-baseline" \
 "n16e8k:150:python bench.py --drones 16 --envs 8192 --no-cpu-baseline" \
 "n16gen:150:python bench.py --config n16 --no-cpu-baseline --drones 16" 
