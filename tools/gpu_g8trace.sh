#!/bin/bash
# Phase timelines of gemm8_kernel (trace build) on the step's shapes.
export LCLIB=exp_so/liblcclip_trace.so
for cfg in "768 3072 0 0" "2304 768 0 0" "3072 768 6 0" "3072 768 7 0" "768 768 0 0"; do
  set -- $cfg
  echo "=== N=$1 K=$2 EPI=$3 FP8=$4"
  for wg in 100 300; do
    N=$1 K=$2 EPI=$3 FP8=$4 WG=$wg timeout -k 10 120 python -u tools/g8_trace.py 2>&1 | grep -v amdgpu
  done
done
