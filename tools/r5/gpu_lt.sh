#!/bin/bash
# r5: LoRA B = 128 step anatomy (kernel trace by shape).
source gpu_step.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_lt
run lt_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lt -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --method lora --batch 128
python tools/trace_by_shape.py gpurun_out/prof_lt/run_kernel_trace.csv 8 45 > gpurun_out/lt_by_shape.txt 2>&1
echo done
