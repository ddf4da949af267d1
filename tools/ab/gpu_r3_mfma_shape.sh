#!/bin/bash
# r3: bf16 MFMA shape (16x16x32 vs 32x32x16) vs the held clock, register-resident loop
# (tools/mfma_shape_clock.hip), random and zero operands.
source gpu_step.sh
B=lifelong-clip_amd/lcclip/ab/mfma_shape_clock
run mshape_rand 120 $B
run mshape_zero 120 $B z
echo done
