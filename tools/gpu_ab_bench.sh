#!/bin/bash
# Headline step A/B: product build vs exp_so/liblcclip_$V.so, three interleaved pairs on one box.
source gpu_step.sh
for r in 1 2 3; do
  run st_prod$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  LCCLIP_LIB=exp_so/liblcclip_$V.so run st_$V$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
echo done
