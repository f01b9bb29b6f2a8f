bash tools/gpu_steps.sh r04m \
 "evvar:600:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vprod vmrot vtinym vprod vmrot vtinym" \
 "parity:300:SWARM_MI355X_LIB=build/var/vmrot.so python -u -m pytest tests/test_gpu_eval.py -q -x --timeout 120 --timeout-method thread"
