#!/bin/bash
# r3 session 2: attention forward in one pass with a running max (LCCLIP_ATTN_FWD_ONLINE=1)
# vs the exact two-pass form, same box.
source gpu_step.sh
export TMPDIR=/tmp
LCCLIP_ATTN_FWD_ONLINE=1 run t_attn_online 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attn or attention"
for r in 1 2; do
  LCCLIP_ATTN_FWD_ONLINE=1 run attn_online_$r 120 python -u tools/bench_attn.py
  run attn_2pass_$r 120 python -u tools/bench_attn.py
done
for r in 1 2; do
  LCCLIP_ATTN_FWD_ONLINE=1 run ad_online_$r 200 python -u bench.py --no-cpu-baseline
  run ad_2pass_$r 200 python -u bench.py --no-cpu-baseline
done
LCCLIP_ATTN_FWD_ONLINE=1 run t_model_online 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py
echo done
