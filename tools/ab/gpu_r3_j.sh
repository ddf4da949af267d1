#!/bin/bash
# r3: attention backward knockouts (timing only): where the 220 us go
source gpu_step.sh
export TMPDIR=/tmp
A=lifelong-clip_amd/lcclip/ab
run attn_full 200 python -u tools/bench_attn.py
for m in ${KOS:-1 2 4 8}; do LCCLIP_LIB=$A/ko$m.so run attn_ko$m 200 python -u tools/bench_attn.py; done
echo done
