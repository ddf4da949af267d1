#!/bin/bash
# Epilogue cost of the 256x256 GEMMs: the product build vs diagnostic builds with the epilogue off
# (make EXTRA_FLAGS=-DG8_NOSTORE=1 OBJDIR=build_ns1 OUT=../../exp_so/liblcclip_NS1.so) or only its
# global stores off (=2, NS2), and the ragged-round cost (M = 49 152).
source gpu_step.sh
for r in 1 2; do
  VARIANTS=8,7 run prod$r 200 python -u tools/bench_gemm.py
  VARIANTS=8,7 LCLIB=exp_so/liblcclip_NS1.so run ns1_$r 200 python -u tools/bench_gemm.py
  VARIANTS=8,7 LCLIB=exp_so/liblcclip_NS2.so run ns2_$r 200 python -u tools/bench_gemm.py
done
M=49152 VARIANTS=8,7 run m49k 200 python -u tools/bench_gemm.py
echo done
