#!/bin/bash
# 4-wave GEMM: DMA distance 3 (tile 7) vs 4 (tile 13) vs gemm8 vs hipBLASLt; step traces
source gpu_step.sh
run c_gemm 300 env VARIANTS=8,7,13,hb REPS=10 python -u tools/bench_gemm.py
for t in 7 13; do
run c_trace_w4_${t}_fc2 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=$t N=768 K=3072 WG=100 python -u tools/w4_trace.py
run c_trace_w4_${t}_qkv 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=$t N=2304 K=768 WG=100 python -u tools/w4_trace.py
done
echo done
