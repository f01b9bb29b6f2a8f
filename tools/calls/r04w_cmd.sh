bash tools/gpu_steps.sh r04w \
 "evvar:600:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vpre vflat vpre vflat vpre vflat" \
 "drv:400:VAR_BENCH_ARGS='--steps 20 --warmup 5' bash tools/run_variants.sh vpre vflat vpre vflat vpre vflat" \
 "k200:400:bash tools/run_variants.sh vpre vflat vpre vflat" \
 "n16:300:VAR_BENCH_ARGS='--config n16 --steps 500 --warmup 50' bash tools/run_variants.sh vpre vflat vpre vflat" \
 "parity:400:python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_step64.py tests/test_gpu_step16.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread"
