#!/bin/bash
# MVP step: product build vs exp_so/liblcclip_$V.so, interleaved.
source gpu_step.sh
for r in 1 2; do
  run mvp_prod$r 300 python -u tools/bench_mvp.py
  LCCLIP_LIB=exp_so/liblcclip_$V.so run mvp_$V$r 300 python -u tools/bench_mvp.py
done
echo done
