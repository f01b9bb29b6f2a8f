bash tools/gpu_steps.sh r04v \
 "rehearsal:700:bash tools/gpu_rehearsal.sh r04v" \
 "suite2:900:python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread -p no:randomly"
