#!/bin/bash
# Round-end evidence: GPU tests + smoke + the bench lines DESIGN cites, then the kernel-trace
# profile and the PMC traffic passes (tools/profile_round.sh) of the default bench.
source gpu_step.sh
rm -f gpurun_out/parity_metrics.jsonl
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench_default 300 python -u bench.py
run bench_c100 300 python -u bench.py --classes 100 --no-cpu-baseline
run bench_lora 300 python -u bench.py --method lora --batch 128 --no-cpu-baseline
run bench_maple 300 python -u tools/bench_maple.py
run bench_mvp 300 python -u tools/bench_mvp.py
TAG=${TAG:-r02_v6} bash tools/profile_round.sh
echo done
