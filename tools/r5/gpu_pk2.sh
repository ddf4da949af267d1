#!/bin/bash
# r5: MVP tests incl. the prompt-row-keep exactness test.
source gpu_step.sh
run pk2_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mvp_gpu.py
