bash tools/gpu_steps.sh r04zg \
 "evtests:600:SWARM_MI355X_LIB=build/var/vev16.so python -u -m pytest tests/test_gpu_eval.py -q -x --timeout 300 --timeout-method thread" \
 "n16ev:400:VAR_BENCH_ARGS='--config n16 --eval --steps 200 --warmup 20' bash tools/run_variants.sh vfin vev16 vfin vev16"
