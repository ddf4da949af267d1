#!/bin/bash
# Quick GPU pass: gpu tests + bench (no profile).
#   gpurun --timeout 600 -- bash tools/gpu_quick.sh
source gpu_step.sh
run tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
