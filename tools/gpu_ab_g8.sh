#!/bin/bash
# A/B of the phase-interleaved GEMM: committed-variant library (exp_so/$OLD) vs the current build,
# interleaved on one box, plus the GEMM correctness tests of the current build.
source gpu_step.sh
run g8tests 300 python -u -m pytest tests/test_fp8_gpu.py "tests/test_kernels_gpu.py::test_gemm_nt_every_tile_exact" "tests/test_kernels_gpu.py::test_gemm_splitk_tail" -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  VARIANTS=8,f8 LCLIB=exp_so/${OLD:-liblcclip_g8a.so} run old$r 300 python -u tools/bench_gemm.py
  VARIANTS=8,f8 run new$r 300 python -u tools/bench_gemm.py
done
echo done
