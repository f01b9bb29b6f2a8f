bash tools/gpu_r03.sh r03b \
 "valu:60:build/valu_rate4" \
 "var:400:bash tools/run_variants.sh base gprio3 gprio1 plev2" \
 "stag6:120:python bench.py --stagger-us 6 --no-cpu-baseline" \
 "stag10:120:python bench.py --stagger-us 10 --no-cpu-baseline" \
 "stag13:120:python bench.py --stagger-us 13 --no-cpu-baseline" \
 "tl_g2:120:SWARM_STAMPS_LIB=build/var/stamps.so python tools/stamps_groups.py 2 200 0" \
 "tl_g2s10:120:SWARM_STAMPS_LIB=build/var/stamps.so python tools/stamps_groups.py 2 200 10" \
 "tl_g1:120:SWARM_STAMPS_LIB=build/var/stamps.so python tools/stamps_groups.py 1 200 0" \
 "reh2:300:SWARM_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --config n256 --gpus 2 --steps 40 --warmup 5 --no-cpu-baseline" \
 "suite:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
