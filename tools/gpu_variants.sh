source gpu_step.sh
VARIANTS=1,2,8 run gv 300 python -u tools/bench_gemm.py
