#!/bin/bash
# adapter + LayerNorm forward with x_out / y staged in LDS and stored as whole rows vs base.so
# (HEAD before it): GPU tests, the kernel alone, the step (interleaved)
source gpu_step.sh
B=lifelong-clip_amd/lcclip/ab/base.so
run w_tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests
run w_adk 120 python -u tools/bench_adapter_kernels.py
run w_adk_base 120 env LCLIB=$B python -u tools/bench_adapter_kernels.py
run w_adk_ko3 120 env LCLIB=lifelong-clip_amd/lcclip/ab/adln_ko3.so python -u tools/bench_adapter_kernels.py
run w_bench 300 python -u bench.py --no-cpu-baseline
run w_bench_base 300 env LCCLIP_LIB=$B python -u bench.py --no-cpu-baseline
run w_bench2 300 python -u bench.py --no-cpu-baseline
run w_bench_base2 300 env LCCLIP_LIB=$B python -u bench.py --no-cpu-baseline
echo done
