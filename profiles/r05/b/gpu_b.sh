#!/bin/bash
# r5: where the one-rank RCCL step loses against the plain step (8151 vs 9403 img/s in gpu_a).
source gpu_step.sh
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
run b_plain 300 $B
LCCLIP_SIDE_STREAMS=1 run b_plain_side1 300 $B
run b_dist 300 $B --force-dist
LCCLIP_SIDE_STREAMS=2 run b_dist_side2 300 $B --force-dist
GPU_MAX_HW_QUEUES=8 run b_dist_q8 300 $B --force-dist
LCCLIP_OVERLAP_GRADS=0 run b_dist_noovl 300 $B --force-dist
run b_plain2 300 $B
grep -h -o '"value": [0-9.]*' gpurun_out/b_*.log
