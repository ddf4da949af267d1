#!/bin/bash
# r5: attention software pipelines, same-box interleaved A/B: base = HEAD (ab/base.so), fwdpipe =
# forward only (ab/fwdpipe.so), new = forward + backward (the working tree's library).
source gpu_step.sh
run f_test 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_f16_gpu.py -k attention
for i in 1 2; do
  LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so run f_attn_base$i 120 python tools/bench_attn.py
  LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/fwdpipe.so run f_attn_fwdpipe$i 120 python tools/bench_attn.py
  run f_attn_new$i 120 python tools/bench_attn.py
done
for i in 1 2; do
  LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so run f_step_base$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run f_step_new$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
grep -H "fwd\|bwd" gpurun_out/f_attn_*.log
grep -Ho '"value": [0-9.]*' gpurun_out/f_step_*.log
