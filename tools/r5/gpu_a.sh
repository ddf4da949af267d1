#!/bin/bash
# r5 first pass: the new tests, split-K under the cross-XCD slice deal, the bench launcher path.
source gpu_step.sh
PY="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
run a_new 600 $PY tests/test_kernels_gpu.py -k "splitk or vit_embed or adapter_bwd_fused or gemm" tests/test_model_gpu.py -k "kept_grad or splitk or vit_embed or adapter_bwd_fused or gemm"
LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/spread.so run a_spread 600 $PY tests/test_kernels_gpu.py -k "splitk or gemm"
run a_launch 300 python bench.py --gpus 1 --force-dist --steps 10 --warmup 3 --no-cpu-baseline
run a_bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
