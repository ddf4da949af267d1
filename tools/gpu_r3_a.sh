#!/bin/bash
# r3: the 2-workgroup GEMM (tile 9) — correctness, then shape timings beside gemm8, then the
# baseline pass (GPU tests, default bench, LoRA bench).
source gpu_step.sh
run gemm_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm"
VARIANTS=8,7,9 run bench_gemm 300 python -u tools/bench_gemm.py
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run bench_default 300 python -u bench.py
run bench_lora 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
echo done
