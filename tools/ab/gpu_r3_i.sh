#!/bin/bash
# r3: attention loops without in-loop mask branches (steady / edge bodies) — parity + same-box
# A/B against the previous build (lcclip/ab/base.so).
source gpu_step.sh
export TMPDIR=/tmp
B=lifelong-clip_amd/lcclip/ab/base.so
run k_tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or attn"
run attn_new 200 python -u tools/bench_attn.py
LCCLIP_LIB=$B run attn_base 200 python -u tools/bench_attn.py
for r in 1 2; do
  run bench_new_$r 300 python -u bench.py --no-cpu-baseline
  LCCLIP_LIB=$B run bench_base_$r 300 python -u bench.py --no-cpu-baseline
done
echo done
