#!/bin/bash
# r5: MaPLe step anatomy: serial (OVERLAP=0) vs overlapped step times and kernel traces of the
# bf16 and fp8 steps.
source gpu_step.sh
export TMPDIR=/tmp
run m2_ovl 300 python tools/bench_maple.py
run m2_ser 300 env OVERLAP=0 python tools/bench_maple.py
mkdir -p gpurun_out/prof_m2b gpurun_out/prof_m2f
run m2_tr 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_m2b -o run -- python tools/bench_maple.py
grep -h ms_per_step gpurun_out/m2_*.log
