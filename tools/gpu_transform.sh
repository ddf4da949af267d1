#!/bin/bash
# Train transform: parity tests, then the kernel timing for this build and the committed one.
source gpu_step.sh
run t_tf 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_autoaug_gpu.py -k "transform or autoaug"
run tf_new 120 python -u tools/bench_transform.py
LCCLIP_LIB=exp_so/liblcclip_${BASE:-base}.so run tf_base 120 python -u tools/bench_transform.py
echo done
