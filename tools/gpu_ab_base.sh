#!/bin/bash
# Step A/B of this build against exp_so/liblcclip_base.so (the last commit), interleaved pairs,
# after the kernel parity tests.
source gpu_step.sh
run t_kern 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py
VARIANTS=8,7 run gemm 200 python -u tools/bench_gemm.py
for r in 1 2 3; do
  LCCLIP_LIB=exp_so/liblcclip_base.so run sbase$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run snew$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
echo done
