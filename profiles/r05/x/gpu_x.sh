#!/bin/bash
# r5: the frozen prompt towers (MVP, MaPLe bf16 / fp8) in the half residual stream (embed cast,
# EPI_RESID16, half-x LayerNorms incl. the fp8 forms; gradient f32): kernel tests, MVP / MaPLe
# parity tests, same-box A/B of both steps.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run x_fp8 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp8_gpu.py
run x_prompt 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_mvp_gpu.py tests/test_maple_gpu.py
cp gpurun_out/parity_metrics.jsonl gpurun_out/x_parity_metrics.jsonl 2>/dev/null
for i in 1 2; do
  run x_mvp32_$i 300 env RESID32=1 python tools/bench_mvp.py
  run x_mvp16_$i 300 python tools/bench_mvp.py
  run x_maple32_$i 300 env RESID32=1 python tools/bench_maple.py
  run x_maple16_$i 300 python tools/bench_maple.py
done
grep -H "ms_per_step" gpurun_out/x_mvp*.log gpurun_out/x_maple*.log
