#!/bin/bash
# r5: attention forward with deferred max raises (threshold 2^8) and the row sums on the MFMA
# (ab/fwd.so), plus the backward with a wave-uniform wave index (the working tree); tests, then
# same-box interleaved A/B against HEAD (ab/base.so), kernels and step.
source gpu_step.sh
run k_test 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_kernels_gpu.py tests/test_f16_gpu.py tests/test_model_gpu.py -k "attention or full_shapes or step_vs_oracle or golden"
for i in 1 2 3; do
  LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so run k_attn_base$i 120 python tools/bench_attn.py
  LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/fwd.so run k_attn_fwd$i 120 python tools/bench_attn.py
  run k_attn_new$i 120 python tools/bench_attn.py
done
for i in 1 2; do
  LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so run k_step_base$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run k_step_new$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
grep -H "image" gpurun_out/k_attn_*.log
grep -Ho '"value": [0-9.]*' gpurun_out/k_step_*.log
