#!/bin/bash
# fp8-output GEMM epilogues: bit-exactness tests, MaPLe fp8 parity, then the MaPLe step with the
# fused epilogues vs LCCLIP_FP8_FUSE=0 (bf16 epilogue + quant_fp8), interleaved on one box.
source gpu_step.sh
run q8tests 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_maple_gpu.py -x -v --timeout 120 --timeout-method thread
for r in 1 2; do
  run mp_fuse$r 300 python -u tools/bench_maple.py
  LCCLIP_FP8_FUSE=0 run mp_nofuse$r 300 python -u tools/bench_maple.py
done
echo done
