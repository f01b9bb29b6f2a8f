bash tools/gpu_steps.sh r04q \
 "polabl:800:VAR_BENCH_ARGS='--policy f32x3 --steps 50 --warmup 5' bash tools/run_variants.sh vprod vclean vxa8 vxa16 vxa32 vxa4 vxa60 vprod vclean vxa8 vxa16 vxa32 vxa4 vxa60" \
 "cleanpar:300:SWARM_MI355X_LIB=build/var/vclean.so python -u -m pytest tests/test_gpu_policy.py -q -x --timeout 120 --timeout-method thread && SWARM_MI355X_LIB=build/var/vclean5.so python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_step64.py -q -x --timeout 120 --timeout-method thread"
bash tools/gpu_steps.sh r04q \
 "g1:120:python bench.py --steps 20 --warmup 5 --groups 1 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g2:120:python bench.py --steps 20 --warmup 5 --groups 2 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g3:120:python bench.py --steps 20 --warmup 5 --groups 3 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g4:120:python bench.py --steps 20 --warmup 5 --groups 4 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g1b:120:python bench.py --steps 20 --warmup 5 --groups 1 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g2b:120:python bench.py --steps 20 --warmup 5 --groups 2 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g3b:120:python bench.py --steps 20 --warmup 5 --groups 3 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g4b:120:python bench.py --steps 20 --warmup 5 --groups 4 --no-cpu-baseline --cpu-variant-seconds 0"
