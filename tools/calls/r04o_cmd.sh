bash tools/gpu_steps.sh r04o \
 "aux200:600:bash tools/run_variants.sh vaux16 vaux0 vaux2 vaux18 vaux17 vaux16 vaux0 vaux2 vaux18 vaux17" \
 "aux20:400:VAR_BENCH_ARGS='--steps 20 --warmup 5' bash tools/run_variants.sh vaux16 vaux2 vaux18 vaux16 vaux2 vaux18"
