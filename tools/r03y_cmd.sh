bash tools/gpu_r03.sh r03y \
 "d1:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "d2:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "def:200:python bench.py" \
 "d3:120:python bench.py --gpus 1 --steps 20 --warmup 5"
