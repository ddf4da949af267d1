#!/bin/bash
# r3 final check of the committed code: the whole GPU suite, smoke and the default bench.
source gpu_step.sh
export TMPDIR=/tmp
rm -f gpurun_out/parity_metrics.jsonl
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench_default 300 python -u bench.py
run bench_maple 300 python -u tools/bench_maple.py
echo done
