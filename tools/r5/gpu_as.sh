#!/bin/bash
# r5 experiment: cache-policy bits on the attention backward's dq|dk|dv stores (nt / sc0+nt):
# attention microbench and same-box step A/B.
source gpu_step.sh
for i in 1 2; do
  for v in prod attst2 attst3; do
    lib=""; [ $v != prod ] && lib=lifelong-clip_amd/lcclip/ab/$v.so
    run as_a_${v}_$i 200 env LCCLIP_LIB=$lib python tools/bench_attn.py
  done
done
for i in 1 2; do
  for v in prod attst2 attst3; do
    lib=""; [ $v != prod ] && lib=lifelong-clip_amd/lcclip/ab/$v.so
    run as_b_${v}_$i 300 env LCCLIP_LIB=$lib python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  done
done
grep -H "image" gpurun_out/as_a_*.log
grep -Ho '"value": [0-9.]*' gpurun_out/as_b_*.log
