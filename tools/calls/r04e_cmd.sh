bash tools/gpu_steps.sh r04e \
 "drvA1:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "drvE1:120:python bench.py --gpus 1 --steps 20 --warmup 5 --events-before 1" \
 "drvA2:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "drvE2:120:python bench.py --gpus 1 --steps 20 --warmup 5 --events-before 1" \
 "drvA3:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "drvE3:120:python bench.py --gpus 1 --steps 20 --warmup 5 --events-before 1" \
 "evvar:300:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vevreg vbase vevreg vbase" \
 "pmcvar:300:bash tools/pmc_variants.sh r04e base_lib vnorowg vnorowgfin" \
 "tests:400:python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_step64.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread" \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread"
