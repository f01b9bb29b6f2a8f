bash tools/gpu_r03.sh r03s \
 "step16:400:python -u -m pytest tests/test_gpu_step16.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread" \
 "n16:150:python bench.py --config n16 --no-cpu-baseline" \
 "n16b:150:python bench.py --config n16 --no-cpu-baseline" \
 "st16:180:SWARM_STAMPS_LIB=build/var/stamps16.so python tools/stamps16.py 1024 60"
