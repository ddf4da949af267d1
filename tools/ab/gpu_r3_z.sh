#!/bin/bash
# r3 session 2: fp8 towers — ln_1's backward writes the next block's c_proj dX operand in fp8
# (ops.layernorm_bwd_fp8) instead of a quant_fp8 pass; vs LCCLIP_FP8_FUSE=3 (the quant_fp8 pass), same box.
source gpu_step.sh
export TMPDIR=/tmp
AB=lifelong-clip_amd/lcclip/ab
run t_fp8 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_fp8_gpu.py tests/test_maple_gpu.py tests/test_kernels_gpu.py -k "fp8 or maple or layernorm"
for r in 1 2; do
  run maple_new_$r 300 python -u tools/bench_maple.py
  LCCLIP_FP8_FUSE=3 run maple_base_$r 300 python -u tools/bench_maple.py
done
run t_model 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_maple_gpu.py tests/test_mvp_gpu.py
echo done
