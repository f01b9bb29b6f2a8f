IC="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
bash tools/gpu_steps.sh r04j \
 "icHead:200:COUNTERS='$IC' bash tools/pmc_variants.sh r04jH vnew" \
 "icEval:200:COUNTERS='$IC' PMC_BENCH_ARGS='--eval --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline --cpu-variant-seconds 0' bash tools/pmc_variants.sh r04jE vnew vevall2" \
 "icN256:200:COUNTERS='$IC' PMC_BENCH_ARGS='--config n256 --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline --cpu-variant-seconds 0' bash tools/pmc_variants.sh r04jN vnew" \
 "icN16:200:COUNTERS='$IC' PMC_BENCH_ARGS='--config n16 --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline --cpu-variant-seconds 0' bash tools/pmc_variants.sh r04jQ vnew" \
 "polvar:400:VAR_BENCH_ARGS='--policy f32x3 --steps 50 --warmup 5' bash tools/run_variants.sh vpipe2 vpipe vpipe2 vpipe" \
 "pol2parity:300:SWARM_MI355X_LIB=build/var/vpipe2.so python -u -m pytest tests/test_gpu_policy.py -q -x --timeout 120 --timeout-method thread"
