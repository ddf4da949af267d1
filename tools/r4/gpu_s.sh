#!/bin/bash
# attention backward: DCE-safe store knockout (stores replaced by keep-alive asm) vs full
source gpu_step.sh
for i in 1 2; do
run s_full_$i 120 python -u tools/bench_attn.py
run s_kost_$i 120 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/att_kost.so python -u tools/bench_attn.py
done
echo done
