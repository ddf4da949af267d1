#!/bin/bash
# r5: M = 12 800 (MaPLe's 64 images) step shapes, tile variants (auto, gemm8, 128x128, 128x64).
source gpu_step.sh
run g12 300 env M=12800 VARIANTS=0,8,1,4 python tools/bench_gemm.py
grep "M=" gpurun_out/g12.log
