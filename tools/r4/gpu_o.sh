#!/bin/bash
# gemm8 split-K slice phases (trace build): slab stores / ticket / reduce / epilogue
source gpu_step.sh
for wg in 600 601 602 603 604 605; do
run o_g8_$wg 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so N=768 K=3072 WG=$wg python -u tools/g8_trace.py
done
echo done
