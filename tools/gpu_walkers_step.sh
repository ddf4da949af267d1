#!/bin/bash
# In-step effect of the PEFT weight-gradient walker count (LC_TN_WALKERS: fewer workgroups, each
# streaming more rows, displace fewer GEMM tiles on the main stream).
source gpu_step.sh
for r in 1 2; do
  for w in 256 128 64 32; do
    LC_TN_WALKERS=$w run w${w}_$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  done
done
echo done
