B="python bench.py --no-cpu-baseline --steps 20 --warmup 5"
bash tools/gpu_r03.sh r03x \
 "g0a:120:$B" "h1a:120:$B --eager-head 1" "h2a:120:$B --eager-head 2" "ea:120:$B --no-graph" \
 "g0b:120:$B" "h1b:120:$B --eager-head 1" "h2b:120:$B --eager-head 2" "eb:120:$B --no-graph" \
 "g0c:120:$B" "h1c:120:$B --eager-head 1" "h2c:120:$B --eager-head 2" "ec:120:$B --no-graph"
