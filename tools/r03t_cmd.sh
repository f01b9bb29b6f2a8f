bash tools/gpu_r03.sh r03t \
 "p1:150:SWARM_MI355X_LIB=build/var/prev.so python bench.py --config n16 --no-cpu-baseline" \
 "c1:150:SWARM_MI355X_LIB=build/var/cur.so python bench.py --config n16 --no-cpu-baseline" \
 "p2:150:SWARM_MI355X_LIB=build/var/prev.so python bench.py --config n16 --no-cpu-baseline" \
 "c2:150:SWARM_MI355X_LIB=build/var/cur.so python bench.py --config n16 --no-cpu-baseline" \
 "st16:180:SWARM_STAMPS_LIB=build/var/stamps16.so python tools/stamps16.py 1024 60"
