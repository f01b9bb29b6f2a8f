bash tools/gpu_steps.sh r04f \
 "bpparity:400:SWARM_MI355X_LIB=build/var/vbperm.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step64.py tests/test_gpu_eval.py -q -x --timeout 120 --timeout-method thread" \
 "bpvar:400:VAR_BENCH_ARGS='--steps 20 --warmup 5' bash tools/run_variants.sh vbperm vbase vbperm vbase vbperm vbase" \
 "bpvar200:300:bash tools/run_variants.sh vbperm vbase vbperm vbase" \
 "bpeval:300:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vbperm vbase" \
 "pmcvar:300:bash tools/pmc_variants.sh r04f vbperm" \
 "evon:200:python bench.py --eval --steps 500 --warmup 50 --no-cpu-baseline --cpu-variant-seconds 0" \
 "evoff:200:python bench.py --groups 2 --no-graph --steps 500 --warmup 50 --no-cpu-baseline --cpu-variant-seconds 0" \
 "ctdeF:200:SWARM_BENCH_FORCE_GATHER=1 python bench.py --config n256 --no-cpu-baseline --cpu-variant-seconds 0" \
 "ctdeN:200:python bench.py --config n256 --no-cpu-baseline --cpu-variant-seconds 0" \
 "ctdeX:200:python bench.py --config n256 --no-ctde --no-cpu-baseline --cpu-variant-seconds 0"
