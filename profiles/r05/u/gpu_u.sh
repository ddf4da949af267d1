#!/bin/bash
# r5: the image tower's residual GRADIENT in half too (scaled, lc_layernorm_bwd_g16 /
# lc_adapter_wgrad_ws_unscaled): kernel tests, model / trainer parity, smoke, same-box step A/B
# against the previous commit (ab/base.so: half residual, f32 gradient) and the f32 stream.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run u_kern 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "x16 or g16 or unscaled or adapter_ln or vit_embed or layernorm or wgrad"
run u_model 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_model_gpu.py tests/test_online_gpu.py tests/test_dp_gpu.py
cp gpurun_out/parity_metrics.jsonl gpurun_out/u_parity_metrics.jsonl 2>/dev/null
run u_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
  run u_step32_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --resid32
  run u_step16_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
export TMPDIR=/tmp
run u_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
python tools/trace_by_shape.py gpurun_out/u_prof/run_kernel_trace.csv 8 40 > gpurun_out/u_by_shape.txt 2>&1
grep -Ho '"value": [0-9.]*' gpurun_out/u_step*.log
head -14 gpurun_out/u_by_shape.txt
