#!/bin/bash
# r3: MaPLe (config 5) bf16 vs fp8 step, and a kernel trace of each precision.
source gpu_step.sh 2>/dev/null || true
export TMPDIR=/tmp
run maple_bench 300 python -u tools/bench_maple.py
P=gpurun_out/prof_maple
PREC=fp8 STEPS=5 WARM=2 run trace_maple_fp8 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/fp8 -o run -- python tools/bench_maple.py
PREC=bf16 STEPS=5 WARM=2 run trace_maple_bf16 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/bf16 -o run -- python tools/bench_maple.py
python tools/trace_by_shape.py $P/fp8/run_kernel_trace.csv 7 45 > gpurun_out/r03_maple_fp8_by_shape.txt 2>&1
python tools/trace_by_shape.py $P/bf16/run_kernel_trace.csv 7 45 > gpurun_out/r03_maple_bf16_by_shape.txt 2>&1
echo done
