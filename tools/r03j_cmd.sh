bash tools/gpu_r03.sh r03j \
 "split:200:SWARM_MI355X_LIB=build/var/a1024.so python bench.py --split-reset --no-cpu-baseline" \
 "nosplit:200:SWARM_MI355X_LIB=build/var/a1024.so python bench.py --no-cpu-baseline" \
 "prof:300:SWARM_MI355X_LIB=build/var/a1024.so rocprofv3 --kernel-trace --stats -d gpurun_out/r03j/prof -o run --output-format csv -- python3 bench.py --split-reset --steps 200 --no-cpu-baseline"
