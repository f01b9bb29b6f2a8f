args=""
for r in 1 2 3; do
  for v in "sr:--graph split --warm-graph ring" "sw:--graph split --warm-graph whole" "fw:--graph fused --warm-graph whole"; do
    n=${v%%:*}; a=${v#*:}
    args="$args \"${n}$r:150:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $a\""
  done
done
args="$args \"fw500:150:python bench.py --graph fused --no-cpu-baseline\" \"gfx:150:python tools/graph_fork_exp.py\""
eval bash tools/gpu_r03.sh r03k $args
