#!/bin/bash
# r5: same-box A/B of the plain N = 1 step at 4 (HIP default) vs 8 hardware queues.
source gpu_step.sh
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2 3; do
  LCCLIP_HW_QUEUES=4 run o_q4_$i 300 $B
  run o_q8_$i 300 $B
done
grep -Ho '"value": [0-9.]*\|"GPU_MAX_HW_QUEUES": "[0-9]*"' gpurun_out/o_*.log
