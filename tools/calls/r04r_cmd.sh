VC="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
bash tools/gpu_steps.sh r04r \
 "vN256:200:COUNTERS='$VC' PMC_BENCH_ARGS='--config n256 --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline --cpu-variant-seconds 0' bash tools/pmc_variants.sh r04rN base_lib" \
 "vHead:200:COUNTERS='$VC' bash tools/pmc_variants.sh r04rH base_lib" \
 "vN16:200:COUNTERS='$VC' PMC_BENCH_ARGS='--config n16 --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline --cpu-variant-seconds 0' bash tools/pmc_variants.sh r04rQ base_lib"
