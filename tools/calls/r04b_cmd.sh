bash tools/gpu_steps.sh r04b \
 "probe:60:./build/anyorder_probe 1 200 8 && ./build/anyorder_probe 512 100 64" \
 "tests:400:python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_ctde.py tests/test_gpu_step16.py tests/test_gpu_eval.py -q -x --timeout 120 --timeout-method thread" \
 "drv:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "drv2:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "def:200:python bench.py" \
 "n256:200:python bench.py --config n256" \
 "n16:200:python bench.py --config n16" \
 "polx3:200:python bench.py --policy f32x3 --steps 50 --warmup 5 --no-cpu-baseline" \
 "evoff:200:python bench.py --groups 2 --no-graph --no-cpu-baseline --cpu-variant-seconds 0" \
 "evon:200:python bench.py --groups 2 --eval --no-cpu-baseline --cpu-variant-seconds 0" \
 "st256:120:SWARM_STAMPS_KERNEL=n256 SWARM_STAMPS_LIB=build/stamps/libswarm_stamps256.so python tools/stamps.py run 1024 256" \
 "q16var:200:VAR_BENCH_ARGS='--config n16 --steps 400 --warmup 20' bash tools/run_variants.sh vq16floor vq16direct vq16w4 vbase" \
 "h256var:200:VAR_BENCH_ARGS='--config n256 --steps 400 --warmup 20' bash tools/run_variants.sh vh256split vbase vh256split vbase" \
 "pmcvar:500:bash tools/pmc_variants.sh r04b base_lib vbase vfin vrow vobs vnores" \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread"
