#!/bin/bash
# r3: 2-WG GEMM variants (9, 10) + the one-pass LoRA gradient: correctness, shape timings,
# LoRA bench and a kernel trace of the LoRA step.
source gpu_step.sh
export TMPDIR=/tmp
run gemm_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or lora"
VARIANTS=8,9,10 run bench_gemm 300 python -u tools/bench_gemm.py
run lora_model 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k "lora"
run bench_lora 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
LCCLIP_LORA_1P=0 run bench_lora_4g 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
P=gpurun_out/prof_lora
run trace_lora 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python bench.py --method lora --batch 128 --steps 5 --warmup 2 --no-cpu-baseline
python tools/trace_by_shape.py $P/trace/run_kernel_trace.csv 8 45 > gpurun_out/r03_lora_by_shape.txt 2>&1
echo done
