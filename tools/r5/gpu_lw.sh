#!/bin/bash
# r5 experiment: the LoRA gradient kernel's walker count (256 = one per CU, 128, 64; diagnostic
# build, LC_LORA_WALKERS) against the step's main-stream GEMMs, LoRA B = 128.
source gpu_step.sh
L=lifelong-clip_amd/lcclip/ab/diag.so
for i in 1 2; do
  for w in 0 128 64; do
    run lw_${w}_$i 300 env LCCLIP_LIB=$L LC_LORA_WALKERS=$w python bench.py --steps 20 --warmup 5 --no-cpu-baseline --method lora --batch 128
  done
done
grep -Ho '"value": [0-9.]*' gpurun_out/lw_*.log
