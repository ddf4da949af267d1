#!/bin/bash
# Tile-raster group size (LC_GEMM_GM) A/B on the step's GEMM shapes (g8 and w4 kernels), with the
# GEMM tests under a grouped raster.
source gpu_step.sh
LC_GEMM_GM=8 run gmtests 300 python -u -m pytest tests/test_fp8_gpu.py "tests/test_kernels_gpu.py::test_gemm_nt_every_tile_exact" "tests/test_kernels_gpu.py::test_gemm_splitk_tail" -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  for gm in 1 4 8 16; do
    LC_GEMM_GM=$gm VARIANTS=8,7 run gm${gm}_$r 200 python -u tools/bench_gemm.py
  done
done
echo done
