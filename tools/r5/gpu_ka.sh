#!/bin/bash
# r5 experiment: HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) on the step benches.
source gpu_step.sh
for i in 1 2; do
  run ka_off_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run ka_on_$i 300 env HIP_FORCE_DEV_KERNARG=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run ka_moff_$i 300 python tools/bench_maple.py
  run ka_mon_$i 300 env HIP_FORCE_DEV_KERNARG=1 python tools/bench_maple.py
done
grep -Ho '"value": [0-9.]*' gpurun_out/ka_o*.log
grep -Ho '"ms_per_step": [0-9.]*' gpurun_out/ka_m*.log
