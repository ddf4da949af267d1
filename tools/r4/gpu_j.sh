#!/bin/bash
# gemm8 (panel mode reverted: no spills) vs 4-wave split-K kernel vs hipBLASLt; step A/B of the
# routing (tile 12 = automatic with the 4-wave kernel in place of gemm8), interleaved
source gpu_step.sh
run j_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k gemm --timeout 120 --timeout-method thread
run j_gemm 400 env VARIANTS=8,7,hb REPS=10 python -u tools/bench_gemm.py
run j_bench_auto 300 python -u bench.py --no-cpu-baseline
run j_bench_w4 300 python -u bench.py --no-cpu-baseline --gemm-tile 12
run j_bench_auto2 300 python -u bench.py --no-cpu-baseline
run j_bench_w4_2 300 python -u bench.py --no-cpu-baseline --gemm-tile 12
echo done
