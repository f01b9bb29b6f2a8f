B="python bench.py --no-cpu-baseline --config n256"
bash tools/gpu_r03.sh r03z "g2:120:$B" "g3:120:$B --groups 3" "g4:120:$B --groups 4" "g1:120:$B --groups 1" "g2b:120:$B"
