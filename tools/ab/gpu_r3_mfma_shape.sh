#!/bin/bash
# r3: bf16 MFMA shape (16x16x32 vs 32x32x16) vs the held clock, register-resident loop
# (tools/mfma_shape_clock.hip), random and zero operands, 2 and 1 waves per SIMD.
source gpu_step.sh
B=lifelong-clip_amd/lcclip/ab/mfma_shape_clock
run mshape_rand 120 $B r 2
run mshape_zero 120 $B z 2
run mshape_rand1 120 $B r 1
run mshape_zero1 120 $B z 1
echo done
