MC="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
bash tools/gpu_steps.sh r04zc \
 "mixE:200:COUNTERS='$MC' PMC_BENCH_ARGS='--eval --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline --cpu-variant-seconds 0' bash tools/pmc_variants.sh r04zcE base_lib" \
 "mixH:200:COUNTERS='$MC' bash tools/pmc_variants.sh r04zcH base_lib"
