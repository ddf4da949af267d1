#!/bin/bash
source gpu_step.sh
for wg in 600 601 602 700 748; do
run l_tr_$wg 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so TILE=7 N=768 K=3072 WG=$wg NS=32 python -u tools/w4_trace.py
done
echo done
