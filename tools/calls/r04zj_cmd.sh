bash tools/gpu_steps.sh r04zj \
 "evtests:600:python -u -m pytest tests/test_gpu_eval.py -q -x --timeout 300 --timeout-method thread"
