bash tools/gpu_r03.sh r03l \
 "pol_bf16:200:python bench.py --policy bf16 --no-cpu-baseline --steps 200" \
 "pol_f32:300:python bench.py --policy f32 --no-cpu-baseline --steps 40 --warmup 5" \
 "prof_bf16:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r03l/prof_bf16 -o run --output-format csv -- python3 bench.py --policy bf16 --no-cpu-baseline --steps 100 --warmup 10" \
 "prof_f32:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r03l/prof_f32 -o run --output-format csv -- python3 bench.py --policy f32 --no-cpu-baseline --steps 20 --warmup 3" \
 "pmc_bf16:120:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r03l/pmc_bf16 -o run -- python3 bench.py --policy bf16 --groups 1 --steps 20 --warmup 3 --device-warmup-ms 0 --no-cpu-baseline" \
 "pmc_f32:120:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r03l/pmc_f32 -o run -- python3 bench.py --policy f32 --groups 1 --steps 10 --warmup 2 --device-warmup-ms 0 --no-cpu-baseline"
