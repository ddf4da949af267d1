#!/bin/bash
# 4-wave GEMM with SRD buffer DMA at distance 4 (tile 13) vs tile 7 / gemm8 / hipBLASLt; knockouts
source gpu_step.sh
run d_gemm 300 env VARIANTS=8,7,13,hb REPS=10 python -u tools/bench_gemm.py
run d_nodma 300 env LCLIB=lifelong-clip_amd/lcclip/ab/nodma.so VARIANTS=7,13 REPS=10 python -u tools/bench_gemm.py
run d_noread 300 env LCLIB=lifelong-clip_amd/lcclip/ab/noread.so VARIANTS=7,13 REPS=10 python -u tools/bench_gemm.py
run d_trace_w4_7 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=7 N=768 K=3072 WG=100 python -u tools/w4_trace.py
run d_trace_w4_13 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=13 N=768 K=3072 WG=100 python -u tools/w4_trace.py
echo done
