#!/bin/bash
# Widened attention output stores (store_row64): attention parity tests, the attention
# microbenchmark and step A/B pairs against the committed build (exp_so/liblcclip_base.so).
source gpu_step.sh
run t_attn 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp8_gpu.py -k "attn or attention"
run ab_new 200 python -u tools/bench_attn.py
LCCLIP_LIB=exp_so/liblcclip_base.so run ab_base 200 python -u tools/bench_attn.py
for r in 1 2 3; do
  LCCLIP_LIB=exp_so/liblcclip_base.so run sbase$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run snew$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
echo done
