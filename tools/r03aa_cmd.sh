B="python bench.py --no-cpu-baseline"
N="python bench.py --no-cpu-baseline --config n256"
D="python bench.py --no-cpu-baseline --steps 20 --warmup 5"
bash tools/gpu_r03.sh r03aa \
 "h2a:120:$B --groups 2" "h4a:120:$B --groups 4" "h2b:120:$B --groups 2" "h4b:120:$B --groups 4" "h3a:120:$B --groups 3" \
 "d2a:120:$D --groups 2" "d4a:120:$D --groups 4" "d2b:120:$D --groups 2" "d4b:120:$D --groups 4" "d3a:120:$D --groups 3" \
 "n4:120:$N --groups 4" "n6:120:$N --groups 6" "n8:120:$N --groups 8" "n4b:120:$N --groups 4"
