#!/bin/bash
# r5: adapter_ln_fwd_x16 standalone with its whole-row stores knocked out (diagnostic builds:
# ADLN_KO 1 = no x_out stores, 2 = no y stores, 3 = neither; results wrong, timing only).
source gpu_step.sh
for i in 1 2; do
  for v in prod ko1 ko2 ko3; do
    lib=""; [ $v != prod ] && lib=lifelong-clip_amd/lcclip/ab/$v.so
    run ko_${v}_$i 120 env LCCLIP_LIB=$lib python tools/bench_adln16.py
  done
done
grep -H "adapter_ln" gpurun_out/ko_*.log
