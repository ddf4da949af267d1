#!/bin/bash
# r4 first pass: GPU tests on the r4 code, baseline bench on this box, vendor-GEMM calibration
# (hipBLASLt through torch.matmul on the same shapes), gemm8 phase traces.
source gpu_step.sh
run a_tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run a_bench 300 python -u bench.py --no-cpu-baseline
run a_gemm_hb 300 env VARIANTS=8,hb SQUARE=1 python -u tools/bench_gemm.py
run a_trace_fc2 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so N=768 K=3072 WG=100 python -u tools/g8_trace.py
run a_trace_qkv 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so N=2304 K=768 WG=100 python -u tools/g8_trace.py
run a_trace_fc1 120 env LCLIB=lifelong-clip_amd/lcclip/ab/trace.so N=3072 K=768 EPI=6 WG=100 python -u tools/g8_trace.py
run a_maple 300 python -u tools/bench_maple.py
run a_maple_seq 300 env OVERLAP=0 python -u tools/bench_maple.py
echo done
