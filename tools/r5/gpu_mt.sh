#!/bin/bash
# r5: MVP (config 3 per-GPU shape) step anatomy: kernel trace by shape.
source gpu_step.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_mt
run mt_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mt -o run -- python tools/bench_mvp.py
python tools/trace_by_shape.py gpurun_out/prof_mt/run_kernel_trace.csv 13 45 > gpurun_out/mt_by_shape.txt 2>&1
echo done
