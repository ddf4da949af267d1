#!/bin/bash
# r3 session 2: raster group size of the 256x256 GEMMs (LC_GEMM_GM row panels per group; default
# 8 for N >= 2304, 1 below) on the step shapes, standalone, same box.
source gpu_step.sh
export TMPDIR=/tmp
for r in 1 2; do
  for gm in 0 2 4 6 12 16; do
    LC_GEMM_GM=$gm VARIANTS=8 run gemm_gm${gm}_$r 200 python -u tools/bench_gemm.py
  done
done
echo done
