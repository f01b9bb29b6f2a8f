bash tools/gpu_r03.sh r03n \
 "g1w4:150:SWARM_MI355X_LIB=build/var/stat.so python bench.py --groups 1 --waves-per-simd 4 --no-cpu-baseline" \
 "g2w2:150:SWARM_MI355X_LIB=build/var/stat.so python bench.py --groups 2 --waves-per-simd 2 --no-cpu-baseline" \
 "g1w2:150:SWARM_MI355X_LIB=build/var/stat.so python bench.py --groups 1 --waves-per-simd 2 --no-cpu-baseline" \
 "g1w6:150:SWARM_MI355X_LIB=build/var/stat.so python bench.py --groups 1 --waves-per-simd 6 --no-cpu-baseline" \
 "base:150:python bench.py --no-cpu-baseline"
