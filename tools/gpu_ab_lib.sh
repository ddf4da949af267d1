#!/bin/bash
# Step A/B: this build vs exp_so/liblcclip_$V.so, interleaved pairs (bench.py, default config).
source gpu_step.sh
for r in 1 2 3; do
  run sprod$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  LCCLIP_LIB=exp_so/liblcclip_$V.so run s$V$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
echo done
