NB="--no-cpu-baseline --cpu-variant-seconds 0"
bash tools/gpu_steps.sh r04y \
 "drv1:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "def:300:python bench.py" \
 "drv2:120:python bench.py --gpus 1 --steps 20 --warmup 5 $NB" \
 "drv3:120:python bench.py --gpus 1 --steps 20 --warmup 5 $NB" \
 "drv4:120:python bench.py --gpus 1 --steps 20 --warmup 5 $NB" \
 "n16:200:python bench.py --config n16 $NB" \
 "n256:200:python bench.py --config n256 $NB" \
 "phys:200:python bench.py --dynamics physics $NB" \
 "evon:200:python bench.py --eval --steps 500 --warmup 50 $NB" \
 "evoff:200:python bench.py --no-graph --steps 500 --warmup 50 $NB" \
 "polbf16:200:python bench.py --policy bf16 --steps 100 --warmup 10 $NB" \
 "polf32:200:python bench.py --policy f32 --steps 50 --warmup 5 $NB" \
 "polx3:200:python bench.py --policy f32x3 --steps 50 --warmup 5 $NB" \
 "trdrv:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r04y/trdrv -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 $NB" \
 "trdef:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r04y/trdef -o run --output-format csv -- python3 bench.py $NB" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread"
