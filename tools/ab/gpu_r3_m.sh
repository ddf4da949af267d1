#!/bin/bash
# r3 session 2: deferred side-stream waits (double-buffered dx_midb / dqkv) and batched LoRA
# merges; the r2-form waits (LCCLIP_SIDE_DEFER=0) interleaved on the same box.
source gpu_step.sh
export TMPDIR=/tmp
run tests_k 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "merge or cast or lora"
run tests_m 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_model_gpu.py tests/test_dp_gpu.py tests/test_online_gpu.py
for r in 1 2; do
  run lora_defer_$r 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
  LCCLIP_SIDE_DEFER=0 run lora_old_$r 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
  run ad_defer_$r 300 python -u bench.py --no-cpu-baseline
  LCCLIP_SIDE_DEFER=0 run ad_old_$r 300 python -u bench.py --no-cpu-baseline
done
echo done
