#!/bin/bash
# r3: split-K for launches under one round of 256x256 tiles (plan_split small: MaPLe's N = 768
# GEMMs at 150 tiles) vs LC_GEMM_SPLITK=2 (that split off), same box.
source gpu_step.sh
export TMPDIR=/tmp
run t_sk 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fp8_gpu.py -k "splitk or fp8"
M=12800 VARIANTS=8,f8 run g_new 300 python -u tools/bench_gemm.py
LC_GEMM_SPLITK=2 M=12800 VARIANTS=8,f8 run g_base 300 python -u tools/bench_gemm.py
for r in 1 2; do
  run maple_new_$r 300 python -u tools/bench_maple.py
  LC_GEMM_SPLITK=2 run maple_base_$r 300 python -u tools/bench_maple.py
done
run t_model 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_maple_gpu.py tests/test_mvp_gpu.py
for r in 1 2; do
  run mvp_new_$r 300 python -u tools/bench_mvp.py
  LC_GEMM_SPLITK=2 run mvp_base_$r 300 python -u tools/bench_mvp.py
done
echo done
