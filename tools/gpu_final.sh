#!/bin/bash
# The driver's round-end commands: GPU tests, smoke, default bench.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python -u bench.py
echo done
