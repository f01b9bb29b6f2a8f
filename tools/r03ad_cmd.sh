D="python bench.py --no-cpu-baseline --steps 20 --warmup 5"
A=()
for i in 1 2 3 4; do A+=("e$i:120:$D" "s$i:120:$D --spin-sync"); done
bash tools/gpu_r03.sh r03ad "${A[@]}"
