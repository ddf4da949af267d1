source gpu_step.sh
run tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
VARIANTS=1,5,7 run bg 200 python -u tools/bench_gemm.py
run bench 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
