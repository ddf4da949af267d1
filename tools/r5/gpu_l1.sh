#!/bin/bash
# r5: adapter_ln_fwd with single-exchange LayerNorm statistics (per-wave mean and squared
# deviations combined pairwise: one barrier less per 16-row block): kernel + model tests,
# same-box step A/B (ab/base.so), kernel trace.
source gpu_step.sh
export TMPDIR=/tmp
rm -f gpurun_out/parity_metrics.jsonl
run l1_kern 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "adapter_ln or x16"
run l1_model 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_model_gpu.py tests/test_f16_gpu.py -k "adapter"
cp gpurun_out/parity_metrics.jsonl gpurun_out/l1_parity_metrics.jsonl 2>/dev/null
for i in 1 2 3; do
  run l1_base_$i 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run l1_new_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
mkdir -p gpurun_out/prof_l1
run l1_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l1 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
grep -Ho '"value": [0-9.]*' gpurun_out/l1_*.log
