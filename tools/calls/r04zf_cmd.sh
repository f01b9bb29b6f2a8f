NB="--no-cpu-baseline --cpu-variant-seconds 0"
bash tools/gpu_steps.sh r04zf \
 "trdrv:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r04zf/trdrv -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 $NB" \
 "trdef:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r04zf/trdef -o run --output-format csv -- python3 bench.py $NB" \
 "treval:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r04zf/treval -o run --output-format csv -- python3 bench.py --eval --steps 200 --warmup 20 $NB" \
 "pmc:600:CONFIGS=headline bash tools/pmc_configs.sh r04zf"
