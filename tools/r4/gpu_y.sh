#!/bin/bash
# kernel traces of the LoRA step (config 4 per-GPU shape) and of MaPLe bf16 / fp8 on the r4 code
source gpu_step.sh
export TMPDIR=/tmp
P=gpurun_out/prof_y
mkdir -p $P
run y_lora_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/lora -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --method lora --batch 128
python tools/trace_by_shape.py $P/lora/run_kernel_trace.csv 8 45 > gpurun_out/y_lora_by_shape.txt 2>&1
for p in bf16 fp8; do
  run y_maple_$p 300 env PREC=$p STEPS=5 WARM=2 rocprofv3 --kernel-trace --output-format csv -d $P/m$p -o run -- python tools/bench_maple.py
  python tools/trace_by_shape.py $P/m$p/run_kernel_trace.csv 7 45 > gpurun_out/y_maple_${p}_by_shape.txt 2>&1
done
echo done
