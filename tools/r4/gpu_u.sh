#!/bin/bash
# gemm8 next-tile L2 prefetch experiment (G8_PREFETCH build) vs production, same box
source gpu_step.sh
run u_gemm 300 env VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run u_gemm_pref 300 env LCLIB=lifelong-clip_amd/lcclip/ab/pref.so VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run u_bench 300 python -u bench.py --no-cpu-baseline
run u_bench_pref 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/pref.so python -u bench.py --no-cpu-baseline
run u_bench2 300 python -u bench.py --no-cpu-baseline
run u_bench_pref2 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/pref.so python -u bench.py --no-cpu-baseline
echo done
