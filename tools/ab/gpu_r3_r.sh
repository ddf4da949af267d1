#!/bin/bash
# r3 session 2: after the branch-free epilogue — c_proj dX on gemm8 vs the 4-wave kernel
# (standalone and in-step), and a kernel trace of the default bench.
source gpu_step.sh
export TMPDIR=/tmp
for r in 1 2; do
  VARIANTS=7,8 run gemm_78_$r 200 python -u tools/bench_gemm.py
done
for r in 1 2; do
  run ad_w4_$r 200 python -u bench.py --no-cpu-baseline
  LC_GEMM_MUL_W4=0 run ad_g8_$r 200 python -u bench.py --no-cpu-baseline
done
P=gpurun_out/prof_s2
mkdir -p $P
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
python tools/trace_by_shape.py $P/run_kernel_trace.csv 8 45 > gpurun_out/s2_by_shape.txt 2>&1
echo done
