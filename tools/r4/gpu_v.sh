#!/bin/bash
# production check (gemm8 + gemm_nt_kernel DMA through buffer descriptors) + gemm8 phase traces
# (SRD code vs the previous global_load_lds code) + same-box A/B vs base.so (HEAD before the
# gemm_nt_kernel change): adapter step, LoRA step, MaPLe
source gpu_step.sh
B=lifelong-clip_amd/lcclip/ab/base.so
run v_tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests
for v in trace trace_old; do
  run v_${v}_fc1 120 env LCLIB=lifelong-clip_amd/lcclip/ab/$v.so N=3072 K=768 EPI=6 python -u tools/g8_trace.py
  run v_${v}_fc2 120 env LCLIB=lifelong-clip_amd/lcclip/ab/$v.so N=768 K=3072 EPI=0 python -u tools/g8_trace.py
done
for v in "" adln_ko1 adln_ko2 adln_ko3; do run v_adk_${v:-prod} 120 env LCLIB=${v:+lifelong-clip_amd/lcclip/ab/$v.so} python -u tools/bench_adapter_kernels.py; done
run v_lora 300 python -u bench.py --no-cpu-baseline --method lora --batch 128
run v_lora_base 300 env LCCLIP_LIB=$B python -u bench.py --no-cpu-baseline --method lora --batch 128
run v_maple 300 python -u tools/bench_maple.py
run v_maple_base 300 env LCCLIP_LIB=$B python -u tools/bench_maple.py
run v_bench 300 python -u bench.py --no-cpu-baseline
run v_bench_base 300 env LCCLIP_LIB=$B python -u bench.py --no-cpu-baseline
run v_lora2 300 python -u bench.py --no-cpu-baseline --method lora --batch 128
run v_lora_base2 300 env LCCLIP_LIB=$B python -u bench.py --no-cpu-baseline --method lora --batch 128
echo done
