#!/bin/bash
# r5: small-M long-K narrow GEMMs (the C = 10 text tower) on 128x64 tiles: GEMM + text-tower
# tests, same-box step A/B (ab/base.so).
source gpu_step.sh
run tw2_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_f16_gpu.py -k "gemm or text"
for i in 1 2 3; do
  run tw2_base_$i 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run tw2_new_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
grep -Ho '"value": [0-9.]*' gpurun_out/tw2_*.log
