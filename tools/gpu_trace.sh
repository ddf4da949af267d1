#!/bin/bash
# rocprofv3 kernel trace of a short bench run + per-(kernel, grid) summary.
#   gpurun --timeout 600 -- bash tools/gpu_trace.sh <tag> [bench args...]
source gpu_step.sh
TAG=${1:-trace}
shift
export TMPDIR=/tmp
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@"
python tools/trace_by_shape.py gpurun_out/prof_$TAG/run_kernel_trace.csv 8 40 > gpurun_out/${TAG}_by_shape.txt 2>&1
python tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_stats.csv 8 40 > gpurun_out/${TAG}_kernel_summary.txt 2>&1
echo done
