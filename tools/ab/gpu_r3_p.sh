#!/bin/bash
# r3 session 2: attention backward with every global access through raw-buffer descriptors
# (range-checked rows, no branches around memory ops -> counted vmcnt, no vmcnt(0) per item)
# vs the dQ-deferral-only build (ab/defer.so) and HEAD (ab/base.so), same box.
source gpu_step.sh
export TMPDIR=/tmp
AB=lifelong-clip_amd/lcclip/ab
run t_attn 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attn or attention"
for r in 1 2; do
  run attn_buf_$r 120 python -u tools/bench_attn.py
  LCCLIP_LIB=$AB/defer.so run attn_defer_$r 120 python -u tools/bench_attn.py
  LCCLIP_LIB=$AB/base.so run attn_base_$r 120 python -u tools/bench_attn.py
done
for r in 1 2; do
  run ad_buf_$r 200 python -u bench.py --no-cpu-baseline
  LCCLIP_LIB=$AB/base.so run ad_base_$r 200 python -u bench.py --no-cpu-baseline
done
run t_model 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_maple_gpu.py tests/test_fp8_gpu.py
echo done
