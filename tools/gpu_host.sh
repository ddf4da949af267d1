source gpu_step.sh
run host 200 python -u tools/host_rate.py
run graph 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph
run eager 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
