#!/bin/bash
# Round check on the GPU box: full GPU test suite, smoke, default bench (the driver's commands).
source gpu_step.sh
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python -u bench.py
echo done
