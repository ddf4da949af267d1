#!/bin/bash
# LayerNorm microbenchmark and headline step: product build vs exp_so/liblcclip_$V.so.
source gpu_step.sh
run lntests 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "layernorm or ln" --timeout 120 --timeout-method thread
for r in 1 2; do
  run ln_prod$r 120 python -u tools/bench_ln.py
  LCCLIP_LIB=exp_so/liblcclip_$V.so run ln_$V$r 120 python -u tools/bench_ln.py
done
for r in 1 2 3; do
  run st_prod$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  LCCLIP_LIB=exp_so/liblcclip_$V.so run st_$V$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
echo done
