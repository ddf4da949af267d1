#!/bin/bash
# New-kernel check: fp8 quantiser + fp8 / bf16 phase-interleaved GEMM parity, then the GEMM
# microbench on the step shapes (pp = 5, w4 = 7, g8 = 8, fp8 = f8).
source gpu_step.sh
run g8tests 300 python -u -m pytest tests/test_fp8_gpu.py "tests/test_kernels_gpu.py::test_gemm_nt_every_tile_exact" "tests/test_kernels_gpu.py::test_gemm_splitk_tail" -x -v --timeout 120 --timeout-method thread
VARIANTS=${VARIANTS:-5,7,8,f8} run bg 300 python -u tools/bench_gemm.py
echo done
