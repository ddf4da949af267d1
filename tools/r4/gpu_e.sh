#!/bin/bash
# 4-wave GEMM step traces with the memory streams knocked out (tile 7, N=768 K=3072)
source gpu_step.sh
for v in trace tr_nodma tr_noread tr_none; do
run e_${v} 120 env LCLIB=lifelong-clip_amd/lcclip/ab/${v}.so TILE=7 N=768 K=3072 WG=100 python -u tools/w4_trace.py
done
echo done
