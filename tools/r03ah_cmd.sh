bash tools/gpu_r03.sh r03ah \
 "s256:600:python -u -m pytest tests/test_gpu_step256.py tests/test_gpu_parity.py -k 'step256 or block or 256' -x -q --timeout 120 --timeout-method thread" \
 "n256:200:python bench.py --config n256 --no-cpu-baseline" \
 "n256b:200:python bench.py --config n256 --no-cpu-baseline"
