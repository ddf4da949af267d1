#!/bin/bash
# GEMM tile rule: 128x128 tiles when they pack a non-splittable ragged round better (vs base.so)
source gpu_step.sh
B=lifelong-clip_amd/lcclip/ab/base.so
run aa_tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests
run aa_bench 300 python -u bench.py --no-cpu-baseline
run aa_bench_base 300 env LCCLIP_LIB=$B python -u bench.py --no-cpu-baseline
run aa_lora 300 python -u bench.py --no-cpu-baseline --method lora --batch 128
run aa_lora_base 300 env LCCLIP_LIB=$B python -u bench.py --no-cpu-baseline --method lora --batch 128
run aa_maple 300 env PREC=bf16 python -u tools/bench_maple.py
run aa_maple_base 300 env PREC=bf16 LCCLIP_LIB=$B python -u tools/bench_maple.py
run aa_bench2 300 python -u bench.py --no-cpu-baseline
run aa_bench_base2 300 env LCCLIP_LIB=$B python -u bench.py --no-cpu-baseline
run aa_lora2 300 python -u bench.py --no-cpu-baseline --method lora --batch 128
run aa_lora_base2 300 env LCCLIP_LIB=$B python -u bench.py --no-cpu-baseline --method lora --batch 128
run aa_maple2 300 env PREC=bf16 python -u tools/bench_maple.py
run aa_maple_base2 300 env PREC=bf16 LCCLIP_LIB=$B python -u tools/bench_maple.py
echo done
