bash tools/gpu_steps.sh r04zi \
 "evtests:600:SWARM_MI355X_LIB=build/var/vevsym.so python -u -m pytest tests/test_gpu_eval.py -q -x --timeout 300 --timeout-method thread" \
 "n256ev:400:VAR_BENCH_ARGS='--config n256 --eval --steps 100 --warmup 10' bash tools/run_variants.sh vprod2 vevsym vprod2 vevsym"
