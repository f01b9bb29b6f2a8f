NB="--no-cpu-baseline --cpu-variant-seconds 0"
bash tools/gpu_steps.sh r04za \
 "ev_n16:200:python bench.py --config n16 --eval --steps 100 --warmup 10 $NB" \
 "ev_g1:200:python bench.py --eval --groups 1 --steps 100 --warmup 10 $NB" \
 "ev_pol:200:python bench.py --eval --policy bf16 --steps 100 --warmup 10 $NB" \
 "x3_n16:200:python bench.py --config n16 --policy f32x3 --steps 50 --warmup 5 $NB" \
 "n256_ev:200:python bench.py --config n256 --eval --steps 50 --warmup 5 $NB" \
 "phys_drv:200:python bench.py --dynamics physics --steps 20 --warmup 5 $NB"
