#!/bin/bash
# r5: the LoRA image tower's residual stream in half (EPI_RESID16 epilogues, half-x LayerNorms;
# its gradient stays f32): GEMM / LN tests, LoRA parity tests, same-box A/B of the LoRA step.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run w_kern 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "resid16 or x16 or g16 or gemm_nt"
run w_model 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_model_gpu.py tests/test_online_gpu.py
cp gpurun_out/parity_metrics.jsonl gpurun_out/w_parity_metrics.jsonl 2>/dev/null
for i in 1 2 3; do
  run w_lora32_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --method lora --batch 128 --resid32
  run w_lora16_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --method lora --batch 128
done
grep -Ho '"value": [0-9.]*\|"image_residual_dtype": "[a-z0-9]*"' gpurun_out/w_lora*.log
