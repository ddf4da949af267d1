#!/bin/bash
# r3 session 2: read traffic (PMC FETCH_SIZE) of the step's GEMM shapes at raster group sizes
# 2 / 8 / 16 row panels (LC_GEMM_GM), to go with the timings of gpu_r3_w.sh.
source gpu_step.sh
export TMPDIR=/tmp
for gm in 2 8 16; do
  LC_GEMM_GM=$gm VARIANTS=8 REPS=2 run fetch_gm$gm 200 timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_gm$gm -o p -- python tools/bench_gemm.py
done
run t_mvp 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_mvp_gpu.py
echo done
