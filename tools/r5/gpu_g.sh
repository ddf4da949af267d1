#!/bin/bash
# r5: the whole GPU suite with the IEEE-half text tower, the parity metrics of the ViT-B/16
# train steps, smoke, bench.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run g_all 1500 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests
cp gpurun_out/parity_metrics.jsonl gpurun_out/g_parity_metrics.jsonl 2>/dev/null
run g_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run g_bench 300 python bench.py --steps 20 --warmup 5
