#!/bin/bash
# fp8 operand fusion (GEMM epilogues, LayerNorm forward, attention backward): bit-exactness tests,
# MaPLe fp8 parity, the MaPLe step per LCCLIP_FP8_FUSE level (3 all ... 0 none), interleaved, and
# the headline step vs exp_so/liblcclip_prev.so (the bf16 attention backward was refactored).
source gpu_step.sh
run q8tests 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_maple_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  for lv in 3 2; do
    LCCLIP_FP8_FUSE=$lv run mp_fuse${lv}_$r 300 python -u tools/bench_maple.py
  done
done
for r in 1 2; do
  run st_new$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  LCCLIP_LIB=exp_so/liblcclip_prev.so run st_prev$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
echo done
