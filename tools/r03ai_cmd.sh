N="python bench.py --config n256 --no-cpu-baseline"
bash tools/gpu_r03.sh r03ai \
 "s256:600:python -u -m pytest tests/test_gpu_step256.py -x -q --timeout 120 --timeout-method thread" \
 "g4:200:$N" "g2:200:$N --groups 2" "g3:200:$N --groups 3" "g4b:200:$N" "g1:200:$N --groups 1"
