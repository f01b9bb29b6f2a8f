bash tools/gpu_r03.sh r03al \
 "tst:600:python -u -m pytest tests/test_gpu_step16.py tests/test_gpu_step256.py -x -q --timeout 120 --timeout-method thread" \
 "n16:150:python bench.py --config n16 --no-cpu-baseline" \
 "n16b:150:python bench.py --config n16 --no-cpu-baseline" \
 "n256:200:python bench.py --config n256 --no-cpu-baseline" \
 "n256b:200:python bench.py --config n256 --no-cpu-baseline" \
 "st16:180:SWARM_STAMPS_LIB=build/var/stamps16.so python tools/stamps16.py 1024 60"
