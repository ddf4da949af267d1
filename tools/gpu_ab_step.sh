#!/bin/bash
# Step A/B: product build vs exp_so/liblcclip_$V.so (LCLIB, read by lcclip._lib), interleaved,
# plus the wgrad microbenchmark of each.
source gpu_step.sh
run wb_prod 200 python -u tools/bench_wgrad.py
LCCLIP_LIB=exp_so/liblcclip_$V.so run wb_$V 200 python -u tools/bench_wgrad.py
for r in 1 2; do
  run st_prod$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  LCCLIP_LIB=exp_so/liblcclip_$V.so run st_$V$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
echo done
