bash tools/gpu_r03.sh r03af \
 "s256:600:python -u -m pytest tests/test_gpu_step256.py -x -q --timeout 120 --timeout-method thread" \
 "blk:600:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_env_cfg.py tests/test_gpu_groups.py tests/test_gpu_ctde.py -x -q --timeout 120 --timeout-method thread" \
 "n256:200:python bench.py --config n256 --no-cpu-baseline" \
 "n256b:200:python bench.py --config n256 --no-cpu-baseline"
