bash tools/gpu_r03.sh r03u \
 "evt:400:python -u -m pytest tests/test_gpu_eval.py -x -q --timeout 120 --timeout-method thread" \
 "evb:150:python tools/eval_bench.py 8192 64 200" \
 "off:150:python bench.py --no-cpu-baseline" \
 "on:150:python bench.py --no-cpu-baseline --eval" \
 "pbf:150:python bench.py --no-cpu-baseline --policy bf16" \
 "pbfe:150:python bench.py --no-cpu-baseline --policy bf16 --eval" \
 "pf32:200:python bench.py --no-cpu-baseline --policy f32 --steps 200" \
 "pf32e:200:python bench.py --no-cpu-baseline --policy f32 --eval --steps 200"
