#!/bin/bash
# r3: streaming fixes (no compiler vmcnt drains) in the fused adapter + LayerNorm and one-pass
# LoRA kernels — parity, adapter / LoRA bench A/Bs, kernel traces of both steps.
source gpu_step.sh
export TMPDIR=/tmp
run k_tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lora or adapter"
run model_tests 600 python -u -m pytest tests/test_model_gpu.py tests/test_online_gpu.py tests/test_mvp_gpu.py tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread
for r in 1 2; do
  run bench_fused_$r 300 python -u bench.py --no-cpu-baseline
  LCCLIP_FUSE_LN=0 run bench_sep_$r 300 python -u bench.py --no-cpu-baseline
done
run bench_lora 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
LCCLIP_LORA_1P=0 run bench_lora_4g 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
P=gpurun_out/prof_adapter
run trace_adapter 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
python tools/trace_by_shape.py $P/trace/run_kernel_trace.csv 8 45 > gpurun_out/r03_adapter_by_shape.txt 2>&1
P=gpurun_out/prof_lora
run trace_lora 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python bench.py --method lora --batch 128 --steps 5 --warmup 2 --no-cpu-baseline
python tools/trace_by_shape.py $P/trace/run_kernel_trace.csv 8 45 > gpurun_out/r03_lora_by_shape.txt 2>&1
echo done
