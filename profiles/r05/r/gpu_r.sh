#!/bin/bash
# r5: row-panel schedule (lc_gemm_set_streamk(4): one workgroup per 256-row panel, 3 column
# tiles each, no cut tiles) for the N = 768 launches vs the split-K tail and hipBLASLt; step A/B.
source gpu_step.sh
run r_test 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "streamk"
run r_gemm 300 env VARIANTS=8,s4,hb python tools/bench_gemm.py
run r_gemm_lora 300 env M=25216 VARIANTS=8,s4 python tools/bench_gemm.py
for i in 1 2; do
  run r_step0_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --streamk 0
  run r_step4_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --streamk 4
done
grep -h "M=" gpurun_out/r_gemm*.log
grep -Ho '"value": [0-9.]*' gpurun_out/r_step*.log
