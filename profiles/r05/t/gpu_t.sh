#!/bin/bash
# r5: the image tower's residual stream in IEEE half (lc_*_x16): kernel tests, the model /
# trainer parity tests, smoke, then a same-box A/B of the step (half vs f32 residual) and a trace.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run t_kern 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "x16 or adapter_ln or vit_embed or layernorm"
run t_model 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_model_gpu.py tests/test_online_gpu.py tests/test_dp_gpu.py
cp gpurun_out/parity_metrics.jsonl gpurun_out/t_parity_metrics.jsonl 2>/dev/null
run t_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
  run t_step32_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --resid32
  run t_step16_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
export TMPDIR=/tmp
run t_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
python tools/trace_by_shape.py gpurun_out/t_prof/run_kernel_trace.csv 8 40 > gpurun_out/t_by_shape.txt 2>&1
grep -Ho '"value": [0-9.]*\|"image_residual_dtype": "[a-z0-9]*"' gpurun_out/t_step*.log
head -16 gpurun_out/t_by_shape.txt
