#!/bin/bash
# rocprofv3 kernel trace of the MaPLe step (PREC=fp8 by default)
mkdir -p gpurun_out
export TMPDIR=/tmp
PREC=${PREC:-fp8} STEPS=5 WARM=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_maple -o run -- python tools/bench_maple.py > gpurun_out/prof_maple.log 2>&1
f=$(find gpurun_out/prof_maple -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" 7 30 > gpurun_out/prof_maple_summary.txt
echo done
