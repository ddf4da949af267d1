#!/bin/bash
# r5: the box exports GPU_MAX_HW_QUEUES=4, which the previous setdefault left in place: bench.py
# now raises it to 8. Same-box A/B at N = 1 (plain and one-rank RCCL) with 4 vs 8 queues.
source gpu_step.sh
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  run n_q8_$i 300 $B
  run n_q8_dist_$i 300 $B --force-dist
done
grep -Ho '"value": [0-9.]*\|"GPU_MAX_HW_QUEUES": "[0-9]*"\|"side_streams": [0-9]' gpurun_out/n_*.log
