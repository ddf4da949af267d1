#!/bin/bash
# Per-round GPU profile of the bench command (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats  -> per-kernel durations (profiles/<round>/kernel_stats.csv)
#   2. --pmc FETCH_SIZE, 3. --pmc WRITE_SIZE (separate passes, MI355X_MICROARCH.md §HBM)
# then tools/pmc_traffic.py turns the counters into per-launch HBM bytes per kernel.
set -e
OUT=gpurun_out/prof_round
export TMPDIR=/tmp
ARGS="bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python $ARGS > $OUT.trace.log 2>&1
echo "trace done"
timeout -k 10 500 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT.fetch.log 2>&1
echo "fetch done"
timeout -k 10 500 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT.write.log 2>&1
echo "write done"
