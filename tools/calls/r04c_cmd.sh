bash tools/gpu_steps.sh r04c \
 "st256:120:SWARM_STAMPS_KERNEL=n256 SWARM_STAMPS_LIB=build/stamps/libswarm_stamps256.so python tools/stamps.py run 1024 256" \
 "drvtrace:200:rocprofv3 --kernel-trace -d gpurun_out/r04c/drvtrace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0" \
 "x3var:300:VAR_BENCH_ARGS='--policy f32x3 --steps 50 --warmup 5' bash tools/run_variants.sh vx3b8 vx3b4late vx3b8" \
 "x3prod:120:python bench.py --policy f32x3 --steps 50 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0" \
 "evvar:300:VAR_BENCH_ARGS='--groups 2 --eval --steps 500 --warmup 50' bash tools/run_variants.sh vevret vevnofe" \
 "evprof:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04c/prof_evon -o run --output-format csv -- python3 bench.py --groups 2 --eval --steps 200 --warmup 10 --no-cpu-baseline --cpu-variant-seconds 0" \
 "q16var:200:VAR_BENCH_ARGS='--config n16 --steps 400 --warmup 20' bash tools/run_variants.sh vq16floor vq16direct vq16w4 vbase" \
 "h256var:200:VAR_BENCH_ARGS='--config n256 --steps 400 --warmup 20' bash tools/run_variants.sh vh256split vbase vh256split vbase" \
 "pmcvar:500:bash tools/pmc_variants.sh r04c base_lib vbase vfin vrow vobs vnores" \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread"
