#!/bin/bash
# r3: fused adapter + LayerNorm forward v2 (double-buffered resid, single z, 2-way K split) —
# parity, bench A/B against the separate launches, kernel trace.
source gpu_step.sh
export TMPDIR=/tmp
run k_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "adapter"
run model_tests 600 python -u -m pytest tests/test_model_gpu.py tests/test_online_gpu.py -x -q --timeout 200 --timeout-method thread
for r in 1 2; do
  run bench_fused_$r 300 python -u bench.py --no-cpu-baseline
  LCCLIP_FUSE_LN=0 run bench_sep_$r 300 python -u bench.py --no-cpu-baseline
done
P=gpurun_out/prof_adapter
run trace_adapter 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
python tools/trace_by_shape.py $P/trace/run_kernel_trace.csv 8 45 > gpurun_out/r03_adapter_by_shape.txt 2>&1
echo done
