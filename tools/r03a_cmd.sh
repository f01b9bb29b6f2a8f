bash tools/gpu_r03.sh r03a \
 "suite:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "driver:200:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "default:200:python bench.py --cpu-variant-seconds 0 --cpu-seconds 3" \
 "var:400:bash tools/run_variants.sh base a1024 a4 a2" \
 "pmc_base:90:SWARM_MI355X_LIB=build/var/base.so rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/r03a/pmc_base -o run -- python3 bench.py --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline" \
 "pmc_a1024:90:SWARM_MI355X_LIB=build/var/a1024.so rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/r03a/pmc_a1024 -o run -- python3 bench.py --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline" \
 "pmc_a4:90:SWARM_MI355X_LIB=build/var/a4.so rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/r03a/pmc_a4 -o run -- python3 bench.py --groups 1 --steps 40 --warmup 5 --device-warmup-ms 0 --no-cpu-baseline"
