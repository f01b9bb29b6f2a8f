bash tools/gpu_steps.sh r04x \
 "evvar:600:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vflat vfebf vflat vfebf vflat vfebf" \
 "evoff:300:VAR_BENCH_ARGS='--no-graph --steps 500 --warmup 50' bash tools/run_variants.sh vflat vflat vflat" \
 "parity:300:SWARM_MI355X_LIB=build/var/vfebf.so python -u -m pytest tests/test_gpu_eval.py -q -x --timeout 120 --timeout-method thread"
