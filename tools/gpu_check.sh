#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench, rocprofv3 kernel-trace summary of the bench.
#   gpurun --timeout 900 -- bash tools/gpu_check.sh [tag]
source gpu_step.sh
TAG=${1:-check}
export TMPDIR=/tmp
run tests 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python -u bench.py --steps 20 --warmup 5
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
STATS=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$STATS" 8 40 > gpurun_out/${TAG}_kernel_summary.txt 2>&1 || true
echo done
