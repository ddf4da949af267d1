#!/bin/bash
# Three-way GEMM A/B: the product build vs exp_so variants ($V1, $V2), interleaved on one box.
source gpu_step.sh
for r in 1 2; do
  VARIANTS=${VARIANTS:-8} run prod$r 200 python -u tools/bench_gemm.py
  VARIANTS=${VARIANTS:-8} LCLIB=exp_so/liblcclip_$V1.so run ${V1}_$r 200 python -u tools/bench_gemm.py
  VARIANTS=${VARIANTS:-8} LCLIB=exp_so/liblcclip_$V2.so run ${V2}_$r 200 python -u tools/bench_gemm.py
done
echo done
