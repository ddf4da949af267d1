#!/bin/bash
# r5: GPU suite + smoke after the golden-oracle fix; same-box A/B of the text tower's storage.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run h_all 1500 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests
cp gpurun_out/parity_metrics.jsonl gpurun_out/h_parity_metrics.jsonl 2>/dev/null
run h_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2; do
  run h_bench_f16_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run h_bench_bf16_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --text-precision bf16
done
grep -Ho '"value": [0-9.]*' gpurun_out/h_bench_*.log
