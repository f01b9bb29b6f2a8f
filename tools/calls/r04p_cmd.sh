bash tools/gpu_steps.sh r04p \
 "evpf:600:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vevp0 vevpf vevp0 vevpf vevp0 vevpf" \
 "evoff:200:VAR_BENCH_ARGS='--groups 2 --no-graph --steps 500 --warmup 50' bash tools/run_variants.sh vevp0 vevp0" \
 "parity:300:SWARM_MI355X_LIB=build/var/vevpf.so python -u -m pytest tests/test_gpu_eval.py -q -x --timeout 120 --timeout-method thread"
