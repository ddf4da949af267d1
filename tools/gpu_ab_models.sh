#!/bin/bash
# MaPLe (both precisions) and MVP step throughput: product build vs exp_so/liblcclip_$V.so.
source gpu_step.sh
for r in 1 2; do
  run mp_prod$r 300 python -u tools/bench_maple.py
  LCCLIP_LIB=exp_so/liblcclip_$V.so run mp_$V$r 300 python -u tools/bench_maple.py
done
run mvp_prod 300 python -u tools/bench_mvp.py
LCCLIP_LIB=exp_so/liblcclip_$V.so run mvp_$V 300 python -u tools/bench_mvp.py
echo done
