#!/bin/bash
# r3: in-kernel clock of gemm8_kernel on the step's shapes (tools/g8_clock.py, clock build), random
# and zero-filled operands, bf16 and fp8; MaPLe bf16/fp8 repeated (s5's single fp8 sample read 5912).
source gpu_step.sh
export TMPDIR=/tmp
L=lifelong-clip_amd/lcclip/ab/clock.so
LCLIB=$L run clock_rand 300 python -u tools/g8_clock.py
ZERO=1 LCLIB=$L run clock_zero 300 python -u tools/g8_clock.py
FP8=1 LCLIB=$L run clock_fp8 300 python -u tools/g8_clock.py
FP8=1 M=12800 LCLIB=$L run clock_fp8_maple 300 python -u tools/g8_clock.py
echo done
