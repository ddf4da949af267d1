#!/bin/bash
# Fused adapter backward knockouts (LC_ADF_DIAG 1: no phase-1 MFMAs, 2: no phase-2 math).
source gpu_step.sh
for d in 0 1 2 0 1 2; do
  LC_ADF_DIAG=$d run akd_$d 120 python -u tools/bench_adapter_kernels.py
done
LC_ADAPTER_FUSED=0 run akd_unf 120 python -u tools/bench_adapter_kernels.py
echo done
