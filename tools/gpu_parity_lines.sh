#!/bin/bash
# Model-level parity tests (logit / gradient bounds of tests/parity.py) and the extra bench lines
# (config 2 at C = 100, LoRA at config 4's per-GPU batch).
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run ptests 600 python -u -m pytest tests/test_model_gpu.py tests/test_mvp_gpu.py tests/test_maple_gpu.py -x -q --timeout 200 --timeout-method thread
run bench_c100 300 python -u bench.py --steps 20 --warmup 5 --classes 100 --no-cpu-baseline
run bench_lora128 300 python -u bench.py --steps 20 --warmup 5 --method lora --batch 128 --no-cpu-baseline
echo done
