#!/bin/bash
# r5: M = 50 432 step shapes, tile variants (auto, gemm8, 128x128, 128x64).
source gpu_step.sh
run g50 300 env VARIANTS=0,8,1,4 python tools/bench_gemm.py
grep "M=" gpurun_out/g50.log
