#!/bin/bash
# r5: C = 100 step anatomy (kernel trace by shape; stream ids in the raw trace).
source gpu_step.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c1
run c1_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c1 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --classes 100
python tools/trace_by_shape.py gpurun_out/prof_c1/run_kernel_trace.csv 8 45 > gpurun_out/c1_by_shape.txt 2>&1
echo done
