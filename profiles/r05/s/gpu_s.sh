#!/bin/bash
# r5: does the stream-K-capable gemm8 (SKM template, modes off) cost the default path anything?
# Same-box interleaved A/B against HEAD's library (ab/base.so): GEMM shapes and the step.
source gpu_step.sh
for i in 1 2; do
  LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so run s_gemm_base$i 300 env VARIANTS=8 python tools/bench_gemm.py
  run s_gemm_new$i 300 env VARIANTS=8 python tools/bench_gemm.py
done
for i in 1 2 3; do
  LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so run s_step_base$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run s_step_new$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
grep -H "M=" gpurun_out/s_gemm*.log
grep -Ho '"value": [0-9.]*' gpurun_out/s_step*.log
