#!/bin/bash
# r5: GPU gradients vs the backward-faithful bf16 oracle (round_bf16_fwd_bwd) at the four
# ViT-B/16 train-step shapes.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run d_steps 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_model_gpu.py -k "step_vs_oracle"
cat gpurun_out/parity_metrics.jsonl
