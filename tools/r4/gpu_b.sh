#!/bin/bash
# hipBLASLt kernel names / resources on the step shapes (kernel trace of torch.matmul);
# model tests + bench after the persistent stack-output gradient pair
source gpu_step.sh
run b_tests 300 python -u -m pytest tests/test_model_gpu.py tests/test_maple_gpu.py tests/test_online_gpu.py -x -q --timeout 120 --timeout-method thread
run b_bench 300 python -u bench.py --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export SQUARE=1 REPS=2
run b_hbtrace 300 env VARIANTS=hb rocprofv3 --kernel-trace --stats -d gpurun_out/hb -o hb --output-format csv -- python3 -u tools/bench_gemm.py
run b_gemm_w4 300 env VARIANTS=8,7,hb REPS=10 python -u tools/bench_gemm.py
echo done
