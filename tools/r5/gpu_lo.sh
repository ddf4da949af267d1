#!/bin/bash
# r5: LoRA B = 128 shapes (M = 25 216): the N = 768 GEMMs' tile routing (1.16 rounds of 256^2
# tiles) — auto (128x64 for K = 768), gemm8, 128x128, and gemm8 with a split-K tail of 4 / 6
# k-tile slices (diagnostic build, LC_GEMM_SPLIT_MIN).
source gpu_step.sh
run lo_g 300 env M=25216 VARIANTS=0,4,8,1 python tools/bench_gemm.py
run lo_s4 300 env M=25216 VARIANTS=8 LCLIB=lifelong-clip_amd/lcclip/ab/diag.so LC_GEMM_SPLIT_MIN=4 python tools/bench_gemm.py
run lo_s6 300 env M=25216 VARIANTS=8 LCLIB=lifelong-clip_amd/lcclip/ab/diag.so LC_GEMM_SPLIT_MIN=6 python tools/bench_gemm.py
cat gpurun_out/lo_g.log gpurun_out/lo_s4.log gpurun_out/lo_s6.log | grep "M="
