#!/bin/bash
# PEFT weight-gradient kernel: tests, standalone timing, step, model tests.
source gpu_step.sh
run wtests 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad or gemm_tn" -x -q --timeout 120 --timeout-method thread
run wbench 200 python -u tools/bench_wgrad.py
run bench 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench2 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
run mtests 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread
echo done
