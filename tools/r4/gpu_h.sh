#!/bin/bash
# same-process A/B: gemm8 auto (panel for N=768 K<=2304) / panel off (14) / panel on (15),
# 4-wave tile 7 vs tile 13 (SRD DMA, distance 4) — tile 13 was never run before (rejected id)
source gpu_step.sh
run h_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k gemm --timeout 120 --timeout-method thread
run h_gemm 400 env VARIANTS=8,14,15,7,13,hb REPS=10 python -u tools/bench_gemm.py
run h_trace_w4_13 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=13 N=768 K=3072 WG=100 python -u tools/w4_trace.py
run h_trace_w4_7 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=7 N=768 K=3072 WG=100 python -u tools/w4_trace.py
echo done
