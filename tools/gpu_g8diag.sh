#!/bin/bash
# Main-loop cost split of the phase-interleaved GEMM: the product build vs diagnostic builds with
# the main-loop DMA (G8_NODMA) or the fragment reads (G8_NOREAD) switched off (wrong results).
source gpu_step.sh
for r in 1 2; do
  VARIANTS=8 run prod$r 200 python -u tools/bench_gemm.py
  VARIANTS=8 LCLIB=exp_so/liblcclip_NODMA.so run nodma$r 200 python -u tools/bench_gemm.py
  VARIANTS=8 LCLIB=exp_so/liblcclip_NOREAD.so run noread$r 200 python -u tools/bench_gemm.py
done
echo done
