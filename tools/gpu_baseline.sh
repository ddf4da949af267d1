#!/bin/bash
# Baseline of the round: GPU tests + default bench + LoRA bench on the box we get.
source gpu_step.sh
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run bench_default 300 python -u bench.py
run bench_lora 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
echo done
