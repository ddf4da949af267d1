#!/bin/bash
# r5 experiment: stagger half of the first-round workgroups of the epilogue-heavy GEMMs
# (gemm8 EPI_GELU_D / EPI_MUL) by 8 / 16 us, so their store-bound epilogues stop coinciding
# across the chip. GEMM microbench and same-box step A/B.
source gpu_step.sh
for lib in "" lifelong-clip_amd/lcclip/ab/stag8.so lifelong-clip_amd/lcclip/ab/stag16.so; do
  n=$(basename "${lib:-prod}" .so)
  run st_g_$n 300 env LCLIB=$lib VARIANTS=8 python tools/bench_gemm.py
done
for i in 1 2; do
  run st_b_prod_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run st_b_s8_$i 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/stag8.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run st_b_s16_$i 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/stag16.so python bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
grep -H "fc1_fwd\|fc2_dx" gpurun_out/st_g_*.log
grep -Ho '"value": [0-9.]*' gpurun_out/st_b_*.log
