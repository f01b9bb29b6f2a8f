bash tools/gpu_r03.sh r03v \
 "g2a:120:python bench.py --no-cpu-baseline --groups 2" \
 "g3a:120:python bench.py --no-cpu-baseline --groups 3" \
 "g4a:120:python bench.py --no-cpu-baseline --groups 4" \
 "g2b:120:python bench.py --no-cpu-baseline --groups 2" \
 "g3b:120:python bench.py --no-cpu-baseline --groups 3" \
 "d2a:120:python bench.py --no-cpu-baseline --groups 2 --steps 20 --warmup 5" \
 "d3a:120:python bench.py --no-cpu-baseline --groups 3 --steps 20 --warmup 5" \
 "d2b:120:python bench.py --no-cpu-baseline --groups 2 --steps 20 --warmup 5" \
 "d3b:120:python bench.py --no-cpu-baseline --groups 3 --steps 20 --warmup 5" \
 "d4a:120:python bench.py --no-cpu-baseline --groups 4 --steps 20 --warmup 5"
