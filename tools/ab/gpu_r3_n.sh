#!/bin/bash
# r3 session 2: split-K slice minimum for the N = K = 768 tail (LC_GEMM_SPLIT_MIN), c_proj dX on
# gemm8 instead of the 4-wave kernel (LC_GEMM_MUL_W4=0), batched LoRA merges
# (LCCLIP_MERGE_BATCH=0: one launch per merge), interleaved on one box; LoRA kernel trace.
source gpu_step.sh
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py"
LC_GEMM_SPLIT_MIN=4 run t_split4 300 $T -k "splitk or merge or epilogues or exact"
LC_GEMM_SPLIT_MIN=6 run t_split6 300 $T -k "splitk"
B="python -u bench.py --no-cpu-baseline"
for r in 1 2; do
  run ad_base_$r 200 $B
  LC_GEMM_MUL_W4=0 run ad_mulg8_$r 200 $B
  LC_GEMM_SPLIT_MIN=6 run ad_split6_$r 200 $B
  LC_GEMM_SPLIT_MIN=4 run ad_split4_$r 200 $B
  run lora_base_$r 200 $B --method lora --batch 128
  LCCLIP_MERGE_BATCH=0 run lora_permerge_$r 200 $B --method lora --batch 128
done
P=gpurun_out/prof_lora
mkdir -p $P
run lora_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --method lora --batch 128
python tools/trace_by_shape.py $P/run_kernel_trace.csv 8 45 > gpurun_out/lora_by_shape.txt 2>&1
echo done
