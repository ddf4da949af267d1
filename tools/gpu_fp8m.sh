#!/bin/bash
source gpu_step.sh
run maple 400 python -u -m pytest tests/test_maple_gpu.py tests/test_fp8_gpu.py -v --timeout 120 --timeout-method thread
run bmaple 300 python -u tools/bench_maple.py
echo done
