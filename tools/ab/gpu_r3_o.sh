#!/bin/bash
# r3 session 2: attention backward with the previous item's dQ rows stored after the next item's
# first barrier (no store latency exposed at the item head) vs HEAD (ab/base.so), same box.
source gpu_step.sh
export TMPDIR=/tmp
BASE=lifelong-clip_amd/lcclip/ab/base.so
run t_attn 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attn or attention"
for r in 1 2; do
  run attn_new_$r 120 python -u tools/bench_attn.py
  LCCLIP_LIB=$BASE run attn_base_$r 120 python -u tools/bench_attn.py
done
for r in 1 2; do
  run ad_new_$r 200 python -u bench.py --no-cpu-baseline
  LCCLIP_LIB=$BASE run ad_base_$r 200 python -u bench.py --no-cpu-baseline
done
run t_model 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_maple_gpu.py
echo done
