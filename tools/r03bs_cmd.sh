bash tools/gpu_r03.sh r03bs \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "def:200:python bench.py" \
 "drv:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "drv2:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "drv3:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "n256:200:python bench.py --config n256" \
 "n16:200:python bench.py --config n16" \
 "prof_drv:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r03bs/prof_drv -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0" \
 "prof_def:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r03bs/prof_def -o run --output-format csv -- python3 bench.py --no-cpu-baseline --cpu-variant-seconds 0" \
 "pmc:900:CONFIGS='headline n256' bash tools/pmc_configs.sh r03bs"
