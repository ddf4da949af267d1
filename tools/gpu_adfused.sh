#!/bin/bash
# One-pass adapter kernels: bit-exactness vs the two-GEMM form, the adapter microbenchmark and
# the headline step with LC_ADAPTER_FUSED=1 (default) vs 0, interleaved on one box.
source gpu_step.sh
run adtests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "adapter" --timeout 120 --timeout-method thread
for f in 1 0 1 0; do
  LC_ADAPTER_FUSED=$f run ak_$f 120 python -u tools/bench_adapter_kernels.py
done
for r in 1 2 3; do
  LC_ADAPTER_FUSED=1 run st_f1_$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  LC_ADAPTER_FUSED=0 run st_f0_$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
echo done
