#!/bin/bash
# r5: the adapter step's out-projections (M = 50 432, N = K = 768) on 128x128 tiles: GEMM tests,
# same-box step A/B against gemm8 for them (ab/base.so).
source gpu_step.sh
run g50b_kern 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm"
for i in 1 2 3; do
  run g50b_base_$i 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run g50b_new_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
grep -Ho '"value": [0-9.]*' gpurun_out/g50b_*.log
