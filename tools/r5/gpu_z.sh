#!/bin/bash
# r5: adapter_ln_fwd_x16 with deeper DMA prefetch (z double-buffered a block ahead, resid
# triple-buffered two blocks ahead): kernel tests, adapter model tests, same-box A/B against the
# previous build (lcclip/ab/base.so), kernel trace of the new build.
source gpu_step.sh
export TMPDIR=/tmp
rm -f gpurun_out/parity_metrics.jsonl
run z_kern 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "adapter_ln or x16 or g16"
run z_model 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_model_gpu.py -k "adapter"
for i in 1 2 3; do
  run z_base_$i 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run z_new_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
mkdir -p gpurun_out/prof_z
run z_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_z -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
grep -Ho '"value": [0-9.]*' gpurun_out/z_*.log
