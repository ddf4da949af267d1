source gpu_step.sh
run tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
VARIANTS=5,5n run bg1 200 python -u tools/bench_gemm.py
LC_GEMM_PERSIST=0 VARIANTS=5,5n run bg0 200 python -u tools/bench_gemm.py
run bench 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
