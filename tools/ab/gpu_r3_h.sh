#!/bin/bash
# r3: fused adapter + LayerNorm forward with both streams double-buffered; persistent attention
# forward — parity, A/Bs, trace; then attention microbench + PMC passes.
source gpu_step.sh
export TMPDIR=/tmp
run k_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "adapter or attention"
run model_tests 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread
run attn_bench_p 200 python -u tools/bench_attn.py
LC_ATTN_FWD_P=0 run attn_bench_i 200 python -u tools/bench_attn.py
for r in 1 2; do
  run bench_new_$r 300 python -u bench.py --no-cpu-baseline
  LC_ATTN_FWD_P=0 run bench_noattnp_$r 300 python -u bench.py --no-cpu-baseline
done
P=gpurun_out/prof_adapter
run trace_adapter 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
python tools/trace_by_shape.py $P/trace/run_kernel_trace.csv 8 45 > gpurun_out/r03_adapter_by_shape.txt 2>&1
run attn_pmc 900 bash tools/pmc_attn.sh
echo done
