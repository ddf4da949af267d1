#!/bin/bash
# Kernel traces of the bench with and without the forced one-rank RCCL exchange (DP overhead).
source gpu_step.sh
export TMPDIR=/tmp
run tr_plain 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dpt_plain -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 run tr_dist 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dpt_dist -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --force-dist
python tools/trace_by_shape.py gpurun_out/dpt_plain/run_kernel_trace.csv 9 40 > gpurun_out/dpt_plain_by_shape.txt 2>&1
python tools/trace_by_shape.py gpurun_out/dpt_dist/run_kernel_trace.csv 9 40 > gpurun_out/dpt_dist_by_shape.txt 2>&1
echo done
