#!/bin/bash
# gemm8 split-K publication with sc1 write-through slabs and no fences vs release/acquire (head)
source gpu_step.sh
run p_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k gemm --timeout 120 --timeout-method thread
for wg in 600 601 602 603; do
run p_g8_$wg 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so N=768 K=3072 WG=$wg python -u tools/g8_trace.py
done
run p_gemm 300 env VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run p_gemm_head 300 env LCLIB=lifelong-clip_amd/lcclip/ab/head.so VARIANTS=8 REPS=10 python -u tools/bench_gemm.py
run p_bench 300 python -u bench.py --no-cpu-baseline
run p_bench_head 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/head.so python -u bench.py --no-cpu-baseline
run p_bench2 300 python -u bench.py --no-cpu-baseline
run p_bench_head2 300 env LCCLIP_LIB=lifelong-clip_amd/lcclip/ab/head.so python -u bench.py --no-cpu-baseline
echo done
