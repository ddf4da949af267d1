#!/bin/bash
# Step A/B: this build vs each exp_so/liblcclip_<V>.so of VS="A B ...", interleaved, 3 rounds.
source gpu_step.sh
for r in 1 2 3; do
  run sprod$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  for v in $VS; do
    LCCLIP_LIB=exp_so/liblcclip_$v.so run s${v}_$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  done
done
echo done
