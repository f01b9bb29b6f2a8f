bash tools/gpu_steps.sh r04z \
 "groups3:400:python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_groups.py -q -x --timeout 120 --timeout-method thread"
