bash tools/gpu_r03.sh r03m \
 "e4k:150:python bench.py --envs 4096 --no-cpu-baseline" \
 "e8k:150:python bench.py --envs 8192 --no-cpu-baseline" \
 "e16k:150:python bench.py --envs 16384 --no-cpu-baseline" \
 "e32k:150:python bench.py --envs 32768 --no-cpu-baseline" \
 "e16kg1:150:python bench.py --envs 16384 --groups 1 --no-cpu-baseline" \
 "e16kg4:150:python bench.py --envs 16384 --groups 4 --no-cpu-baseline"
