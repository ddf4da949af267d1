source gpu_step.sh
for t in 0 2 4; do LC_GEMM_TILE=$t run adk$t 100 python -u tools/bench_adapter_kernels.py; done
echo done
