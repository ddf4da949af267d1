#!/bin/bash
# The RCCL (nccl backend) data-parallel path at world size 1 on the one-GPU box: the DP GPU tests
# and the bench through torch.distributed.run with the process group forced on.
source gpu_step.sh
run dptests 300 python -u -m pytest tests/test_dp_gpu.py -x -q --timeout 200 --timeout-method thread
run bench_dist 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --force-dist --steps 20 --warmup 5 --no-cpu-baseline

run bench_plain 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
