#!/bin/bash
# Full GPU pass for the round profile v10: tests, smoke, bench (with the CPU baseline), rocprofv3
# kernel trace of the bench, separate FETCH_SIZE / WRITE_SIZE PMC passes -> gemm traffic.
source gpu_step.sh
export TMPDIR=/tmp
run tests 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python -u bench.py --steps 20 --warmup 5
mkdir -p gpurun_out/prof_round
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_round/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run fetch 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_round/fetch -o p -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline
run write 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_round/write -o p -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline
python tools/pmc_traffic.py gpurun_out/prof_round/fetch gpurun_out/prof_round/write gpurun_out/gemm_traffic_v10.json > gpurun_out/pmc.log 2>&1
python tools/prof_summary.py gpurun_out/prof_round/trace/run_kernel_stats.csv 8 40 > gpurun_out/v10_kernel_summary.txt 2>&1
python tools/trace_by_shape.py gpurun_out/prof_round/trace/run_kernel_trace.csv 8 40 > gpurun_out/v10_by_shape.txt 2>&1
echo done
