#!/bin/bash
# 4-wave GEMM with split-K tail (tile 7) vs gemm8 (auto / no panel) vs hipBLASLt
source gpu_step.sh
run i_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k gemm --timeout 120 --timeout-method thread
run i_gemm 400 env VARIANTS=8,14,7,hb REPS=10 python -u tools/bench_gemm.py
run i_trace_w4 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=7 N=768 K=3072 WG=100 python -u tools/w4_trace.py
run i_trace_w4_qkv 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=7 N=2304 K=768 WG=100 python -u tools/w4_trace.py
echo done
