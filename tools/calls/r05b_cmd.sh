# VALU-issue test: extra independent f32 muls (2-cycle class) / u32 min-max (4-cycle class) per wave
bash tools/gpu_steps.sh r05b \
 "h64:600:VAR_BENCH_ARGS='--steps 400 --warmup 20' bash tools/run_variants.sh xbase xf256 xi256 xf512 xi512 xbase xf512 xi512" \
 "h256:400:VAR_BENCH_ARGS='--config n256 --steps 400 --warmup 20' bash tools/run_variants.sh hbase hf512 hi512 hbase hf512 hi512"
