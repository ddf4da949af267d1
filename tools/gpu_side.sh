#!/bin/bash
# DP overhead at N = 1 vs the number of HIP hardware queues per process.
source gpu_step.sh
export MASTER_ADDR=127.0.0.1
GPU_MAX_HW_QUEUES=8 run p_q8 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
GPU_MAX_HW_QUEUES=8 MASTER_PORT=29551 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 run d_q8 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --force-dist
MASTER_PORT=29552 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 run d_q4 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --force-dist
run p_q4 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
