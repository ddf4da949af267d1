#!/bin/bash
# r3 session 2: first-round stagger of every other gemm8 workgroup (LC_GEMM_STAGGER x ~3.4 us)
# — do the CUs' epilogue store bursts coincide now that the stores stay in flight?
source gpu_step.sh
export TMPDIR=/tmp
for r in 1 2; do
  for st in 0 2 4 6; do
    LC_GEMM_STAGGER=$st VARIANTS=8 run gemm_st${st}_$r 200 python -u tools/bench_gemm.py
  done
done
for r in 1 2; do
  run ad_st0_$r 200 python -u bench.py --no-cpu-baseline
  LC_GEMM_STAGGER=4 run ad_st4_$r 200 python -u bench.py --no-cpu-baseline
done
echo done
