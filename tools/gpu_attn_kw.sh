#!/bin/bash
# Attention backward at L = 197: 16 keys per wave (14 waves) vs 32 (7 waves), plus the
# attention and model parity tests on the new default.
source gpu_step.sh
run attn_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -q --timeout 120 --timeout-method thread
run kw16 200 python -u tools/bench_attn.py
LC_ATTN_BWD_KW=32 run kw32 200 python -u tools/bench_attn.py
run kw16b 200 python -u tools/bench_attn.py
run mtests 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread
run bench 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
