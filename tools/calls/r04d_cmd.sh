bash tools/gpu_steps.sh r04d \
 "bperm:60:rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d gpurun_out/r04d/bperm -o run -- ./build/bperm_probe" \
 "drvA1:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "drvB1:120:HSA_ENABLE_INTERRUPT=0 python bench.py --gpus 1 --steps 20 --warmup 5" \
 "drvA2:120:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "drvB2:120:HSA_ENABLE_INTERRUPT=0 python bench.py --gpus 1 --steps 20 --warmup 5" \
 "hiptrace:200:rocprofv3 --hip-trace --kernel-trace -d gpurun_out/r04d/hiptrace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0" \
 "evon:200:python bench.py --eval --no-cpu-baseline --cpu-variant-seconds 0" \
 "evoff:200:python bench.py --groups 2 --no-graph --no-cpu-baseline --cpu-variant-seconds 0" \
 "n16:200:python bench.py --config n16 --no-cpu-baseline --cpu-variant-seconds 0" \
 "polx3:200:python bench.py --policy f32x3 --steps 50 --warmup 5 --no-cpu-baseline --cpu-variant-seconds 0" \
 "tests:400:python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_step16.py tests/test_gpu_policy.py -q -x --timeout 120 --timeout-method thread" \
 "suite:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread"
