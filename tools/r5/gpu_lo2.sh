#!/bin/bash
# r5: ragged N = 768, K = 768 GEMMs (LoRA / MVP at 128 images) routed to 128x128 tiles: GEMM
# and model tests, same-box step A/B against the previous routing (ab/base.so).
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run lo2_kern 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm"
run lo2_model 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_model_gpu.py tests/test_mvp_gpu.py -k "lora or mvp"
for i in 1 2 3; do
  run lo2_lb_$i 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline --method lora --batch 128
  run lo2_ln_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --method lora --batch 128
done
for i in 1 2; do
  run lo2_mb_$i 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so python tools/bench_mvp.py
  run lo2_mn_$i 300 python tools/bench_mvp.py
done
grep -Ho '"value": [0-9.]*' gpurun_out/lo2_l*.log
grep -Ho '"ms_per_step": [0-9.]*' gpurun_out/lo2_m*.log
