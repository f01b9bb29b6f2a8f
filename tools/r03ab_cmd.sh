D="python bench.py --no-cpu-baseline --steps 20 --warmup 5"
bash tools/gpu_r03.sh r03ab \
 "e2a:120:$D" "g4a:120:$D --graph-short --groups 4" "f4a:120:$D --graph-short --groups 4 --graph fused" "g2a:120:$D --graph-short" \
 "e2b:120:$D" "g4b:120:$D --graph-short --groups 4" "f4b:120:$D --graph-short --groups 4 --graph fused" "g2b:120:$D --graph-short"
