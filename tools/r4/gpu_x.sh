#!/bin/bash
# gemm8: phase 1's B fragments read in phase 0's LOAD part (G8_EARLYB build, eb.so) vs production
source gpu_step.sh
E=lifelong-clip_amd/lcclip/ab/eb.so
run x_tests_eb 300 env LCCLIP_LIB=$E python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fp8_gpu.py -k "gemm or fp8"
run x_gemm 300 env VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run x_gemm_eb 300 env LCLIB=$E VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run x_bench 300 python -u bench.py --no-cpu-baseline
run x_bench_eb 300 env LCCLIP_LIB=$E python -u bench.py --no-cpu-baseline
run x_bench2 300 python -u bench.py --no-cpu-baseline
run x_bench_eb2 300 env LCCLIP_LIB=$E python -u bench.py --no-cpu-baseline
echo done
