#!/bin/bash
# r3: tile variants on the step's GEMM shapes (out-projection's ragged third round: 256x128 / 128x128
# tiles vs the 256x256 kernel), random data, interleaved rounds.
source gpu_step.sh
export TMPDIR=/tmp
VARIANTS=1,2,4,8 REPS=20 run tiles 300 python -u tools/bench_gemm.py
echo done
