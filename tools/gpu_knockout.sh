source gpu_step.sh
run b0 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
LC_DIAG_SKIP_WGRAD=1 run b_skipw 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline

run b1 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
