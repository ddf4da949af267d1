#!/bin/bash
# r5 experiment: the step on a high-priority HIP stream (side streams at the default priority),
# so that waiting main-stream workgroups are dispatched ahead of side-stream ones.
source gpu_step.sh
for i in 1 2 3; do
  run pr_off_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run pr_on_$i 300 env LCCLIP_MAIN_PRIO=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
for i in 1 2; do
  run pr_loff_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --method lora --batch 128
  run pr_lon_$i 300 env LCCLIP_MAIN_PRIO=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --method lora --batch 128
done
grep -Ho '"value": [0-9.]*' gpurun_out/pr_*.log
