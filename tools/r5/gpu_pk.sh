#!/bin/bash
# r5: MVP prompt rows kept across consecutive prompt layers of one prompt count (no compact /
# expand copies between them): MVP tests, same-box A/B of the config-3 step.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run pk_tests 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_mvp_gpu.py
cp gpurun_out/parity_metrics.jsonl gpurun_out/pk_parity_metrics.jsonl 2>/dev/null
for i in 1 2 3; do
  run pk_off_$i 300 env LCCLIP_PROMPT_KEEP=0 python tools/bench_mvp.py
  run pk_on_$i 300 python tools/bench_mvp.py
done
grep -Ho '"ms_per_step": [0-9.]*' gpurun_out/pk_o*.log
