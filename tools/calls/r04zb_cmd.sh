NB="--no-cpu-baseline --cpu-variant-seconds 0"
bash tools/gpu_steps.sh r04zb \
 "on3:200:python bench.py --eval --groups 3 --steps 500 --warmup 50 $NB" \
 "off3:200:python bench.py --no-graph --groups 3 --steps 500 --warmup 50 $NB" \
 "on4:200:python bench.py --eval --groups 4 --steps 500 --warmup 50 $NB" \
 "off4:200:python bench.py --no-graph --groups 4 --steps 500 --warmup 50 $NB" \
 "on3b:200:python bench.py --eval --groups 3 --steps 500 --warmup 50 $NB" \
 "off3b:200:python bench.py --no-graph --groups 3 --steps 500 --warmup 50 $NB" \
 "on4b:200:python bench.py --eval --groups 4 --steps 500 --warmup 50 $NB" \
 "off4b:200:python bench.py --no-graph --groups 4 --steps 500 --warmup 50 $NB"
