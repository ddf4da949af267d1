#!/bin/bash
# r5: MVP's embed through the fused half-stream embed kernel (and layer 0's ln_1 for the key
# query): MVP tests, same-box A/B (FUSE_EMBED=0: conv1 rows -> assemble -> ln_pre -> cast).
source gpu_step.sh
run me_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mvp_gpu.py
for i in 1 2 3; do
  run me_off_$i 300 env FUSE_EMBED=0 python tools/bench_mvp.py
  run me_on_$i 300 python tools/bench_mvp.py
done
grep -Ho '"ms_per_step": [0-9.]*\|"query_pass_ms": [0-9.]*' gpurun_out/me_o*.log
