#!/bin/bash
# r5: MaPLe prompt learner on the text stream (one stream per leaf): tests (warning gone?),
# same-box A/B of the step against the r4 form (LEARNER_SIDE=0).
source gpu_step.sh
run j_test 600 python -u -m pytest -q -W error::UserWarning --timeout 300 --timeout-method thread tests/test_maple_gpu.py
for i in 1 2 3; do
  LEARNER_SIDE=0 run j_maple_r4_$i 300 python tools/bench_maple.py
  run j_maple_new_$i 300 python tools/bench_maple.py
done
grep -H "ms" gpurun_out/j_maple_*.log | cut -c1-300
