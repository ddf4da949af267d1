#!/bin/bash
# r5: text-tower GEMM shapes (W = 512) at C = 100 (M = 7700) and C = 10 (M = 770): tile variants.
source gpu_step.sh
run tw_7700 300 env M=7700 W=512 VARIANTS=0,1,4 python tools/bench_gemm.py
run tw_770 300 env M=770 W=512 VARIANTS=0,1,4 python tools/bench_gemm.py
grep -h "M=" gpurun_out/tw_*.log
