source gpu_step.sh
PY="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run t_new2 900 $PY tests/test_f16_gpu.py tests/test_dp_gpu.py tests/test_maple_gpu.py tests/test_mvp_gpu.py
run t_maple 300 python -u tools/bench_maple.py
