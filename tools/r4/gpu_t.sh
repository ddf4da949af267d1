#!/bin/bash
# MaPLe: overlap on/off, deep-text-prompt views on/off (regression hunt: 10.16 -> 11.98 ms bf16)
source gpu_step.sh
run t_maple 300 python -u tools/bench_maple.py
run t_maple_noviews 300 env VIEWS=0 python -u tools/bench_maple.py
run t_maple_seq 300 env OVERLAP=0 python -u tools/bench_maple.py
run t_maple2 300 python -u tools/bench_maple.py
echo done
