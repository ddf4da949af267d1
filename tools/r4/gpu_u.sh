#!/bin/bash
# gemm8 experiments vs production, same box: next-tile L2 prefetch (G8_PREFETCH build, pref.so)
# and buffer-descriptor DMA (G8_SRD build, srd.so)
source gpu_step.sh
run u_tests_srd 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/srd.so python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fp8_gpu.py -k "gemm or fp8"
run u_gemm 300 env VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run u_gemm_srd 300 env LCLIB=lifelong-clip_amd/lcclip/ab/srd.so VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run u_gemm_pref 300 env LCLIB=lifelong-clip_amd/lcclip/ab/pref.so VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run u_lora 120 python -u tools/bench_lora_grad.py
run u_bench 300 python -u bench.py --no-cpu-baseline
run u_bench_srd 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/srd.so python -u bench.py --no-cpu-baseline
run u_bench_pref 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/pref.so python -u bench.py --no-cpu-baseline
run u_bench2 300 python -u bench.py --no-cpu-baseline
run u_bench_srd2 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/srd.so python -u bench.py --no-cpu-baseline
run u_bench_pref2 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/pref.so python -u bench.py --no-cpu-baseline
echo done
