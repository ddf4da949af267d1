#!/bin/bash
# A/B of gemm8_kernel's phase count (LC_G8_PH=4 vs 2) on one build, with the GEMM correctness
# tests run under LC_G8_PH=2.
source gpu_step.sh
LC_G8_PH=2 run ph2tests 300 python -u -m pytest tests/test_fp8_gpu.py "tests/test_kernels_gpu.py::test_gemm_nt_every_tile_exact" "tests/test_kernels_gpu.py::test_gemm_splitk_tail" -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  LC_G8_PH=4 VARIANTS=8,f8 run ph4_$r 300 python -u tools/bench_gemm.py
  LC_G8_PH=2 VARIANTS=8,f8 run ph2_$r 300 python -u tools/bench_gemm.py
done
echo done
