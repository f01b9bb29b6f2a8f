bash tools/gpu_r03.sh r03e \
 "var:500:bash tools/run_variants.sh base a4 a2048 a6144 a1024" \
 "g1:120:python bench.py --groups 1 --no-cpu-baseline" \
 "g1w6:120:python bench.py --groups 1 --waves-per-simd 6 --no-cpu-baseline" \
 "g1w4:120:python bench.py --groups 1 --waves-per-simd 4 --no-cpu-baseline" \
 "g3:120:python bench.py --groups 3 --no-cpu-baseline" \
 "g2:120:python bench.py --no-cpu-baseline"
