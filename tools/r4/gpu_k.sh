#!/bin/bash
# 4-wave kernel: split-K tail (7) vs none (13) vs gemm8; traces of a full tile and a tail slice
source gpu_step.sh
run k_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm and (tile or splitk)" --timeout 120 --timeout-method thread
run k_gemm 400 env VARIANTS=8,7,13,hb REPS=10 python -u tools/bench_gemm.py
run k_tr_full 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=7 N=768 K=3072 WG=100 python -u tools/w4_trace.py
run k_tr_tail 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=7 N=768 K=3072 WG=600 NS=32 python -u tools/w4_trace.py
run k_tr_tail2 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=7 N=768 K=3072 WG=748 NS=32 python -u tools/w4_trace.py
echo done
