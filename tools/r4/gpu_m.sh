#!/bin/bash
# gemm8 split-K tail slices: time from loop end to epilogue end (incl. slab publish + reduce)
source gpu_step.sh
for wg in 100 600 601 602 603; do
run m_g8_$wg 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so N=768 K=3072 WG=$wg python -u tools/g8_trace.py
done
echo done
