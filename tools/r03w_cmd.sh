bash tools/gpu_r03.sh r03w \
 "ga:120:python bench.py --no-cpu-baseline --steps 20 --warmup 5" \
 "ea:120:python bench.py --no-cpu-baseline --steps 20 --warmup 5 --no-graph" \
 "gb:120:python bench.py --no-cpu-baseline --steps 20 --warmup 5" \
 "eb:120:python bench.py --no-cpu-baseline --steps 20 --warmup 5 --no-graph" \
 "gc:120:python bench.py --no-cpu-baseline --steps 20 --warmup 5" \
 "ec:120:python bench.py --no-cpu-baseline --steps 20 --warmup 5 --no-graph" \
 "e500:120:python bench.py --no-cpu-baseline --no-graph"
