PB="--policy f32x3 --steps 20 --warmup 2 --device-warmup-ms 0 --no-cpu-baseline --cpu-variant-seconds 0"
bash tools/gpu_steps.sh r04h \
 "evvar:400:VAR_BENCH_ARGS='--eval --steps 500 --warmup 50' bash tools/run_variants.sh vevnone vevtiny vevall2 vevnone vevtiny vevall2" \
 "polvar:300:VAR_BENCH_ARGS='--policy f32x3 --steps 50 --warmup 5' bash tools/run_variants.sh vx3p14 vx3m vx3p14 vx3m" \
 "pmcA:200:COUNTERS='SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE' PMC_BENCH_ARGS='$PB' bash tools/pmc_variants.sh r04hA vx3m" \
 "pmcB:200:COUNTERS='SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT' PMC_BENCH_ARGS='$PB' bash tools/pmc_variants.sh r04hB vx3m" \
 "pmcC:200:COUNTERS='TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum' PMC_BENCH_ARGS='$PB' bash tools/pmc_variants.sh r04hC vx3m" \
 "parity:300:SWARM_MI355X_LIB=build/var/vevtiny.so python -u -m pytest tests/test_gpu_eval.py -q -x --timeout 120 --timeout-method thread"
