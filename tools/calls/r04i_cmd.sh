bash tools/gpu_steps.sh r04i \
 "var20:400:VAR_BENCH_ARGS='--steps 20 --warmup 5' bash tools/run_variants.sh vnew vkeep vbase vnew vkeep vbase" \
 "var200:400:bash tools/run_variants.sh vnew vkeep vbase vnew vkeep vbase" \
 "pmcvar:300:bash tools/pmc_variants.sh r04i vnew vkeep" \
 "n16:300:VAR_BENCH_ARGS='--config n16 --steps 500 --warmup 50' bash tools/run_variants.sh vnew vbase vnew vbase" \
 "n256:300:VAR_BENCH_ARGS='--config n256 --steps 200 --warmup 20' bash tools/run_variants.sh vnew vbase vnew vbase" \
 "evon:400:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vnew vkeep vbase vnew vkeep vbase" \
 "evoff:300:VAR_BENCH_ARGS='--groups 2 --no-graph --steps 500 --warmup 50' bash tools/run_variants.sh vnew vkeep vbase" \
 "keepparity:300:SWARM_MI355X_LIB=build/var/vkeep.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_step64.py tests/test_gpu_eval.py -q -x --timeout 120 --timeout-method thread" \
  "polvar:400:VAR_BENCH_ARGS='--policy f32x3 --steps 50 --warmup 5' bash tools/run_variants.sh vpipe vpipe4 vpipe0 vpipe vpipe4 vpipe0" \
 "polparity:300:SWARM_MI355X_LIB=build/var/vpipe.so python -u -m pytest tests/test_gpu_policy.py -q -x --timeout 120 --timeout-method thread" \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread"
