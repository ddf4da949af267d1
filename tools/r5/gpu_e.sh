#!/bin/bash
# r5: the IEEE-half text tower — f16 kernels, model steps vs the bf16/f16 oracle, then the
# whole GPU suite.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
PY="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
run e_f16 600 $PY tests/test_f16_gpu.py
run e_steps 900 $PY tests/test_model_gpu.py -k "step_vs_oracle or full_shapes or kept_grad or golden or module_path or staging or graph"
cp gpurun_out/parity_metrics.jsonl gpurun_out/e_parity_metrics.jsonl 2>/dev/null
run e_all 1200 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests
run e_bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
