bash tools/gpu_steps.sh r04l \
 "evabl:600:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vprod ve1 ve2 ve4 ve8 ve7 vprod ve1 ve2 ve4 ve8 ve7" \
 "evoff:200:VAR_BENCH_ARGS='--groups 2 --no-graph --steps 500 --warmup 50' bash tools/run_variants.sh vprod vprod" \
 "pmccfg:900:bash tools/pmc_configs.sh r04l"
