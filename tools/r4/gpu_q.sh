#!/bin/bash
# 4-wave kernel (SRD DMA 4 steps ahead, XCD-grouped sc1 split-K tail) for the K-long N = 768
# shapes: microbench vs gemm8, step A/B (--gemm-tile 12 routes those shapes to it)
source gpu_step.sh
run q_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k gemm --timeout 120 --timeout-method thread
run q_gemm 300 env VARIANTS=8,7,hb REPS=10 python -u tools/bench_gemm.py
run q_bench 300 python -u bench.py --no-cpu-baseline
run q_bench_w4 300 python -u bench.py --no-cpu-baseline --gemm-tile 12
run q_bench2 300 python -u bench.py --no-cpu-baseline
run q_bench_w4_2 300 python -u bench.py --no-cpu-baseline --gemm-tile 12
echo done
