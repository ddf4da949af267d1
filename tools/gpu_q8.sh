#!/bin/bash
# fp8 operand fusion (GEMM epilogues, LayerNorm forward): bit-exactness tests, MaPLe fp8 parity,
# then the MaPLe step per LCCLIP_FP8_FUSE level (2 all, 1 GEMM epilogues, 0 none), interleaved.
source gpu_step.sh
run q8tests 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_maple_gpu.py -x -v --timeout 120 --timeout-method thread
for r in 1 2; do
  for lv in 2 1 0; do
    LCCLIP_FP8_FUSE=$lv run mp_fuse${lv}_$r 300 python -u tools/bench_maple.py
  done
done
echo done
