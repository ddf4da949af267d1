#!/bin/bash
# r5: the full GPU suite, smoke and the default bench on the final code.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run fin_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run fin_smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
run fin_bench 300 python -u bench.py
grep -Ho '"value": [0-9.]*' gpurun_out/fin_bench.log
