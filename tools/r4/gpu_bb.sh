#!/bin/bash
# gemm8 with two phases of 32 MFMAs per k-tile (G8_2PH build, g2ph.so) vs production
source gpu_step.sh
E=lifelong-clip_amd/lcclip/ab/g2ph.so
run bb_tests 300 env LCCLIP_LIB=$E python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fp8_gpu.py -k "gemm or fp8"
run bb_gemm 300 env VARIANTS=8,f8 REPS=10 python -u tools/bench_gemm.py
run bb_gemm_2ph 300 env LCLIB=$E VARIANTS=8,f8 REPS=10 python -u tools/bench_gemm.py
run bb_bench 300 python -u bench.py --no-cpu-baseline
run bb_bench_2ph 300 env LCCLIP_LIB=$E python -u bench.py --no-cpu-baseline
run bb_bench2 300 python -u bench.py --no-cpu-baseline
run bb_bench_2ph2 300 env LCCLIP_LIB=$E python -u bench.py --no-cpu-baseline
echo done
