#!/bin/bash
# gemm8 phase traces with the main-loop memory work knocked out (diagnostic builds): full, no
# DMA, no fragment reads, neither — the floor of the two-group barrier structure
source gpu_step.sh
for v in trace tr_nodma tr_noread tr_none; do
  run z_${v}_fc2 120 env LCLIB=lifelong-clip_amd/lcclip/ab/$v.so N=768 K=3072 EPI=0 python -u tools/g8_trace.py
done
run z_gemm25 300 env M=25216 VARIANTS=0,1,2,4,8,hb REPS=10 python -u tools/bench_gemm.py
run z_gemm12 300 env M=12800 VARIANTS=0,1,2,4,8,hb REPS=10 python -u tools/bench_gemm.py
S=lifelong-clip_amd/lcclip/ab/att_st.so
run z_tests_st 300 env LCCLIP_LIB=$S python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attn or attention or model"
run z_attn 120 python -u tools/bench_attn.py
run z_attn_st 120 env LCCLIP_LIB=$S python -u tools/bench_attn.py
run z_bench 300 python -u bench.py --no-cpu-baseline
run z_bench_st 300 env LCCLIP_LIB=$S python -u bench.py --no-cpu-baseline
run z_bench2 300 python -u bench.py --no-cpu-baseline
run z_bench_st2 300 env LCCLIP_LIB=$S python -u bench.py --no-cpu-baseline
echo done
