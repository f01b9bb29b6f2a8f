D="python bench.py --no-cpu-baseline --steps 20 --warmup 5"
A=()
for i in 1 2 3 4 5 6; do A+=("e$i:120:$D" "g$i:120:$D --graph-short"); done
bash tools/gpu_r03.sh r03ac "${A[@]}"
