#!/bin/bash
# r5: head_logits with four classes per wave in flight (MVP's B = 128, C = 200 head): head
# kernel tests, MVP tests, same-box A/B of the config-3 step.
source gpu_step.sh
run hl_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "head" tests/test_mvp_gpu.py
for i in 1 2 3; do
  run hl_base_$i 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/base.so python tools/bench_mvp.py
  run hl_new_$i 300 python tools/bench_mvp.py
done
grep -Ho '"ms_per_step": [0-9.]*' gpurun_out/hl_*.log
