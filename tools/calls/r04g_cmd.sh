bash tools/gpu_steps.sh r04g \
 "pmcvar:300:bash tools/pmc_variants.sh r04g vl128 vl128bp" \
 "var200:400:bash tools/run_variants.sh vl128 vl128bp vbase vl128 vl128bp vbase" \
 "var20:400:VAR_BENCH_ARGS='--steps 20 --warmup 5' bash tools/run_variants.sh vl128 vl128bp vbase vl128 vl128bp vbase" \
 "evvar:300:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vevall vbase vevall vbase" \
 "polvar:400:VAR_BENCH_ARGS='--policy f32x3 --steps 50 --warmup 5' bash tools/run_variants.sh vx3m vx3p6 vbase vx3m vx3p6 vbase" \
 "ctdeN2:200:python bench.py --config n256 --groups 2 --no-graph --no-cpu-baseline --cpu-variant-seconds 0" \
 "ctdeX2:200:python bench.py --config n256 --groups 2 --no-graph --no-ctde --no-cpu-baseline --cpu-variant-seconds 0" \
 "parity:400:SWARM_MI355X_LIB=build/var/vl128.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step64.py -q -x --timeout 120 --timeout-method thread && SWARM_MI355X_LIB=build/var/vl128bp.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step64.py -q -x --timeout 120 --timeout-method thread && SWARM_MI355X_LIB=build/var/vevall.so python -u -m pytest tests/test_gpu_eval.py -q -x --timeout 120 --timeout-method thread && SWARM_MI355X_LIB=build/var/vx3p6.so python -u -m pytest tests/test_gpu_policy.py -q -x --timeout 120 --timeout-method thread && SWARM_MI355X_LIB=build/var/vx3m.so python -u -m pytest tests/test_gpu_policy.py -q -x --timeout 120 --timeout-method thread"
