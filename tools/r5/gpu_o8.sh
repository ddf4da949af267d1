#!/bin/bash
# r5: the out-projection on the fp8 GEMM in fp8 mode (MaPLe config 5): MaPLe parity tests and
# a same-box A/B of the fp8 step (LCCLIP_FP8_OUT=0: out-proj in bf16).
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run o8_tests 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_maple_gpu.py tests/test_fp8_gpu.py
cp gpurun_out/parity_metrics.jsonl gpurun_out/o8_parity_metrics.jsonl 2>/dev/null
for i in 1 2 3; do
  run o8_off_$i 300 env PREC=fp8 LCCLIP_FP8_OUT=0 python tools/bench_maple.py
  run o8_on_$i 300 env PREC=fp8 python tools/bench_maple.py
done
grep -h ms_per_step gpurun_out/o8_o*.log | cut -c1-160
