#!/bin/bash
# r5: the LoRA image tower's residual gradient in half (lc_layernorm_bwd_g16 +
# lc_lora_grad_ws_unscaled): kernel tests, LoRA parity tests, same-box A/B of the LoRA step
# (LCCLIP_HALF_GRAD=0: half stream, f32 gradient).
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run y_kern 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "lora or resid16 or x16 or g16"
run y_model 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_model_gpu.py tests/test_online_gpu.py
cp gpurun_out/parity_metrics.jsonl gpurun_out/y_parity_metrics.jsonl 2>/dev/null
for i in 1 2 3; do
  run y_lora32g_$i 300 env LCCLIP_HALF_GRAD=0 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --method lora --batch 128
  run y_lora16g_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --method lora --batch 128
done
run y_adapter 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
grep -Ho '"value": [0-9.]*' gpurun_out/y_*.log
