#!/bin/bash
# r3: PEFT weight gradients on the side stream (default) vs on the main stream right after their
# producers (LCCLIP_OVERLAP_GRADS=0), adapter and LoRA steps, interleaved on one box.
source gpu_step.sh
export TMPDIR=/tmp
for r in 1 2; do
  run ad_side_$r 300 python -u bench.py --no-cpu-baseline
  LCCLIP_OVERLAP_GRADS=0 run ad_main_$r 300 python -u bench.py --no-cpu-baseline
  run lora_side_$r 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
  LCCLIP_OVERLAP_GRADS=0 run lora_main_$r 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
done
echo done
