NB="--no-cpu-baseline --cpu-variant-seconds 0"
bash tools/gpu_steps.sh r04u \
 "evon:200:python bench.py --eval --steps 500 --warmup 50 $NB" \
 "evoff:200:python bench.py --no-graph --steps 500 --warmup 50 $NB" \
 "evon2:200:python bench.py --eval --steps 500 --warmup 50 $NB" \
 "evoff2:200:python bench.py --no-graph --steps 500 --warmup 50 $NB" \
 "pmccfg:900:bash tools/pmc_configs.sh r04u"
