#!/bin/bash
# Attention backward: tests, microbenchmark, model tests, bench.
source gpu_step.sh
run attn_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -q --timeout 120 --timeout-method thread
run attnb 200 python -u tools/bench_attn.py
run mtests 600 python -u -m pytest tests/test_model_gpu.py tests/test_maple_gpu.py tests/test_mvp_gpu.py -x -q --timeout 200 --timeout-method thread
run bench 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
