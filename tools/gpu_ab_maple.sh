#!/bin/bash
# MaPLe (BASELINE config 5) A/B: this build vs exp_so/liblcclip_$V.so, interleaved, bf16 + fp8.
source gpu_step.sh
for r in 1 2 3; do
  run mprod$r 200 python -u tools/bench_maple.py
  LCCLIP_LIB=exp_so/liblcclip_$V.so run m$V$r 200 python -u tools/bench_maple.py
done
echo done
