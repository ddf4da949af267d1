#!/bin/bash
# r5: stream-K schedule of the 256x256 GEMM (lc_gemm_set_streamk): GEMM tests (new + split-K
# regression), standalone shapes vs the split-K tail and hipBLASLt, step A/B per mode.
source gpu_step.sh
run q_test 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm"
run q_gemm 300 env VARIANTS=8,s2,s3,hb python tools/bench_gemm.py
run q_gemm_lora 300 env M=25216 VARIANTS=8,s2,s3 python tools/bench_gemm.py
for i in 1 2; do
  run q_step0_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --streamk 0
  run q_step1_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --streamk 1
  run q_step2_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --streamk 2
done
grep -h "M=" gpurun_out/q_gemm*.log
grep -Ho '"value": [0-9.]*' gpurun_out/q_step*.log
