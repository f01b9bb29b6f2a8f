bash tools/gpu_steps.sh r04s \
 "g2_0:120:python bench.py --steps 20 --warmup 5 --groups 2 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g3_0:120:python bench.py --steps 20 --warmup 5 --groups 3 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g2_1:120:python bench.py --steps 20 --warmup 5 --groups 2 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g3_1:120:python bench.py --steps 20 --warmup 5 --groups 3 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g2_2:120:python bench.py --steps 20 --warmup 5 --groups 2 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g3_2:120:python bench.py --steps 20 --warmup 5 --groups 3 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g2_3:120:python bench.py --steps 20 --warmup 5 --groups 2 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g3_3:120:python bench.py --steps 20 --warmup 5 --groups 3 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g2_4:120:python bench.py --steps 20 --warmup 5 --groups 2 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g3_4:120:python bench.py --steps 20 --warmup 5 --groups 3 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g2_5:120:python bench.py --steps 20 --warmup 5 --groups 2 --no-cpu-baseline --cpu-variant-seconds 0" \
 "g3_5:120:python bench.py --steps 20 --warmup 5 --groups 3 --no-cpu-baseline --cpu-variant-seconds 0"
VC="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
bash tools/gpu_steps.sh r04s \
 "vN256:200:COUNTERS='$VC' PMC_BENCH_ARGS='--config n256 --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline --cpu-variant-seconds 0' bash tools/pmc_variants.sh r04sN base_lib" \
 "vHead:200:COUNTERS='$VC' bash tools/pmc_variants.sh r04sH base_lib" \
 "vN16:200:COUNTERS='$VC' PMC_BENCH_ARGS='--config n16 --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline --cpu-variant-seconds 0' bash tools/pmc_variants.sh r04sQ base_lib"
