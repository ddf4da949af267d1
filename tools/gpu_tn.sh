#!/bin/bash
# gemm_tn workspace path (LoRA dA / dB): kernel + model tests, the LoRA bench line, and the
# GEMM tile variants at the MaPLe shapes (text M = 7700, image M = 12800).
source gpu_step.sh
run tntests 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_tn or wgrad" -x -q --timeout 120 --timeout-method thread
run lora_tests 600 python -u -m pytest tests/test_model_gpu.py -k "lora" -x -q --timeout 300 --timeout-method thread
run bench_lora 300 python -u bench.py --steps 20 --warmup 5 --method lora --batch 128 --no-cpu-baseline
M=7700 VARIANTS=1,2,4,8 run m7700 200 python -u tools/bench_gemm.py
M=12800 VARIANTS=1,2,4,8 run m12800 200 python -u tools/bench_gemm.py
echo done
