#!/bin/bash
# MaPLe fp8 with the text tower's frozen GEMMs on fp8 too (default now) vs TEXT_FP8=0; tests
source gpu_step.sh
run ee_tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_maple_gpu.py tests/test_fp8_gpu.py
run ee_mt 300 env PREC=fp8 python -u tools/bench_maple.py
run ee_m 300 env PREC=fp8 TEXT_FP8=0 python -u tools/bench_maple.py
run ee_mt2 300 env PREC=fp8 python -u tools/bench_maple.py
run ee_m2 300 env PREC=fp8 TEXT_FP8=0 python -u tools/bench_maple.py
run ee_b 300 env PREC=bf16 python -u tools/bench_maple.py
echo done
