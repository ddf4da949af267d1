#!/bin/bash
# Nontemporal epilogue stores (-DG8_NTST build in exp_so) vs the product build, step shapes.
source gpu_step.sh
for r in 1 2; do
  VARIANTS=8,7 run prod$r 200 python -u tools/bench_gemm.py
  VARIANTS=8,7 LCLIB=exp_so/liblcclip_NT.so run nt$r 200 python -u tools/bench_gemm.py
done
echo done
