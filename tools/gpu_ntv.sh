#!/bin/bash
# Which GEMM outputs to store nontemporally: this build (every bf16 epilogue output) vs NTV1
# (the c_fc QuickGELU output, read at once by c_proj, temporal) and NTV2 (only QuickGELU', read
# in the backward, nontemporal). Interleaved step pairs.
source gpu_step.sh
for r in 1 2 3; do
  run sprod$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  for v in NTV1 NTV2; do
    LCCLIP_LIB=exp_so/liblcclip_$v.so run s${v}_$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  done
done
echo done
