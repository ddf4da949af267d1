#!/bin/bash
# split-K for K = 768 tails (6-k-tile slices) now that the fixup is cheaper: diag build,
# LC_GEMM_SPLIT_MIN=6 vs the default 8
source gpu_step.sh
run r_gemm_min8 300 env LCLIB=lifelong-clip_amd/lcclip/ab/diag.so VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run r_gemm_min6 300 env LCLIB=lifelong-clip_amd/lcclip/ab/diag.so LC_GEMM_SPLIT_MIN=6 VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run r_gemm_min4 300 env LCLIB=lifelong-clip_amd/lcclip/ab/diag.so LC_GEMM_SPLIT_MIN=4 VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run r_bench_min8 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/diag.so python -u bench.py --no-cpu-baseline
run r_bench_min6 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/diag.so LC_GEMM_SPLIT_MIN=6 python -u bench.py --no-cpu-baseline
run r_bench_min8b 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/diag.so python -u bench.py --no-cpu-baseline
run r_bench_min6b 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/diag.so LC_GEMM_SPLIT_MIN=6 python -u bench.py --no-cpu-baseline
echo done
