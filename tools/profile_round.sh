#!/bin/bash
# Round profile of the bench command on the GPU box (run from the repo root):
#   TAG=r02_v1 [TESTS=1] bash tools/profile_round.sh
#   1. (TESTS=1) GPU tests, smoke, default bench (the driver's commands)
#   2. rocprofv3 --kernel-trace --stats of the bench -> <TAG>_kernel_summary.txt, <TAG>_by_shape.txt
#   3. separate --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (MI355X_MICROARCH.md: never combined
#      with other tracing) -> <TAG>_gemm_traffic.json via tools/pmc_traffic.py
# Outputs land in gpurun_out/; copy the ones to keep into profiles/<round>/.
source gpu_step.sh
export TMPDIR=/tmp
TAG=${TAG:-prof}
P=gpurun_out/prof_$TAG
mkdir -p $P
if [ "${TESTS:-0}" = "1" ]; then
  run tests 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
  run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
run bench 400 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-}
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run fetch 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $P/fetch -o p -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline
run write 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $P/write -o p -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline
python tools/pmc_traffic.py $P/fetch $P/write gpurun_out/${TAG}_gemm_traffic.json > gpurun_out/${TAG}_pmc.log 2>&1
python tools/prof_summary.py $P/trace/run_kernel_stats.csv 8 40 > gpurun_out/${TAG}_kernel_summary.txt 2>&1
python tools/trace_by_shape.py $P/trace/run_kernel_trace.csv 8 40 > gpurun_out/${TAG}_by_shape.txt 2>&1
cp $P/trace/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
echo done
