#!/bin/bash
# r3: attention microbench + PMC passes (counters of the current fwd / bwd kernels)
source gpu_step.sh
export TMPDIR=/tmp
run attn_bench 200 python -u tools/bench_attn.py
run attn_pmc 900 bash tools/pmc_attn.sh
echo done
