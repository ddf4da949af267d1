#!/bin/bash
# r3 session 2: GEMM epilogue stores through range-checked buffer descriptors (no row-guard
# branch -> no vmcnt(0) per row group) + attention backward buffer ops, vs HEAD (ab/base.so).
source gpu_step.sh
export TMPDIR=/tmp
AB=lifelong-clip_amd/lcclip/ab
run t_kern 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fp8_gpu.py
for r in 1 2; do
  VARIANTS=8 run gemm_new_$r 200 python -u tools/bench_gemm.py
  VARIANTS=8 LCLIB=$AB/base.so run gemm_base_$r 200 python -u tools/bench_gemm.py
done
run t_attn 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attn or attention"
for r in 1 2; do
  run attn_new_$r 120 python -u tools/bench_attn.py
  LCCLIP_LIB=$AB/base.so run attn_base_$r 120 python -u tools/bench_attn.py
done
for r in 1 2; do
  run ad_new_$r 200 python -u bench.py --no-cpu-baseline
  LCCLIP_LIB=$AB/attn.so run ad_attn_$r 200 python -u bench.py --no-cpu-baseline
  LCCLIP_LIB=$AB/base.so run ad_base_$r 200 python -u bench.py --no-cpu-baseline
  run lora_new_$r 200 python -u bench.py --no-cpu-baseline --method lora --batch 128
  LCCLIP_LIB=$AB/base.so run lora_base_$r 200 python -u bench.py --no-cpu-baseline --method lora --batch 128
done
run maple_new 300 python -u tools/bench_maple.py
LCCLIP_LIB=$AB/base.so run maple_base 300 python -u tools/bench_maple.py
run t_model 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_maple_gpu.py tests/test_mvp_gpu.py tests/test_online_gpu.py
echo done
