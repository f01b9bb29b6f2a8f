bash tools/gpu_steps.sh r04n \
 "polabl:600:VAR_BENCH_ARGS='--policy f32x3 --steps 50 --warmup 5' bash tools/run_variants.sh vprod vxa1 vxa2 vxa3 vxa4 vprod vxa1 vxa2 vxa3 vxa4"
