bash tools/gpu_steps.sh r04zd \
 "parity:300:SWARM_MI355X_LIB=build/var/vfe2.so python -u -m pytest tests/test_gpu_eval.py -q -x --timeout 120 --timeout-method thread" \
 "evvar:700:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vflat vfe2 vflat vfe2 vflat vfe2 vflat vfe2" \
 "evoff:300:VAR_BENCH_ARGS='--no-graph --steps 500 --warmup 50' bash tools/run_variants.sh vflat vflat"
