#!/bin/bash
# gemm8 panel mode (N = 768: one workgroup per row panel) vs the tile grid + split-K tail
source gpu_step.sh
run g_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k gemm --timeout 120 --timeout-method thread
run g_gemm 300 env VARIANTS=8,hb REPS=10 python -u tools/bench_gemm.py
run g_gemm_nopanel 300 env LCLIB=lifelong-clip_amd/lcclip/ab/diag.so LC_GEMM_PANEL=0 VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run g_bench_panel 300 python -u bench.py --no-cpu-baseline
run g_bench_nopanel 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/diag.so LC_GEMM_PANEL=0 python -u bench.py --no-cpu-baseline
run g_bench_panel2 300 python -u bench.py --no-cpu-baseline
echo done
