#!/bin/bash
# r5: MVP's pool gathers (e-prompts, masks) with a GEMM backward instead of torch's sort-based
# index_put accumulate: MVP tests and a same-box A/B of the config-3 step.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run mp_tests 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_mvp_gpu.py
cp gpurun_out/parity_metrics.jsonl gpurun_out/mp_parity_metrics.jsonl 2>/dev/null
for i in 1 2 3; do
  run mp_off_$i 300 env LCCLIP_POOL_GEMM=0 python tools/bench_mvp.py
  run mp_on_$i 300 python tools/bench_mvp.py
done
grep -Ho '"ms_per_step": [0-9.]*' gpurun_out/mp_o*.log
