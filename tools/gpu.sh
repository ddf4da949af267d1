#!/bin/bash
# The one GPU-box entry point (run from the repo root, e.g. through gpurun):
#   bash tools/gpu.sh STEP [STEP ...]
# Each STEP runs under its own time limit (gpu_step.sh: logs in gpurun_out/<name>.log, the
# sequence stops at the first crash / timeout). Steps:
#   tests            the whole `-m gpu` suite (the driver's command)
#   tests:<args>     pytest with <args> (e.g. tests:tests/test_f16_gpu.py)
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (the driver's command)
#   lines            the other bench lines DESIGN quotes: C = 100, LoRA B = 128, the fp16 image
#                    tower, MaPLe (bf16 / fp8), MVP
#   ab:<n>           <n> interleaved pairs of bench runs, the working tree vs the library in
#                    $AB_LIB (LCCLIP_LIB; build it with tools/build_ab.sh), $AB_ENV applied to
#                    the B runs instead when AB_LIB is empty
#   profile          rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the bench
#                    (tools/profile_round.sh, TAG=$TAG)
#   mfma             the MFMA-busy counter pass (tools/gpu_mfma_pmc.sh)
#   round            tests smoke bench lines profile mfma (the round-end evidence)
source gpu_step.sh
export TMPDIR=/tmp
PY="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
step() {
  case "$1" in
    tests) rm -f gpurun_out/parity_metrics.jsonl
           run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ;;
    tests:*) run tests_sel 900 $PY ${1#tests:} ;;
    smoke) run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench_default 300 python -u bench.py ;;
    lines) run bench_c100 300 $B --classes 100
           run bench_lora 300 $B --method lora --batch 128
           run bench_fp16 300 $B --image-precision fp16
           run bench_maple 300 python -u tools/bench_maple.py
           run bench_mvp 300 python -u tools/bench_mvp.py ;;
    ab:*) for i in $(seq 1 ${1#ab:}); do
            run ab_a$i 300 $B
            if [ -n "$AB_LIB" ]; then LCCLIP_LIB=$AB_LIB run ab_b$i 300 $B
            else env $AB_ENV bash -c "source gpu_step.sh; run ab_b$i 300 $B"; fi
          done
          grep -Ho '"value": [0-9.]*\|"ms_fwd_bwd": [0-9.]*' gpurun_out/ab_*.log ;;
    profile) TAG=${TAG:-prof} bash tools/profile_round.sh ;;
    mfma) bash tools/gpu_mfma_pmc.sh ;;
    round) for s in tests smoke bench lines profile mfma; do step $s; done ;;
    *) echo "unknown step $1"; exit 2 ;;
  esac
}
for s in "$@"; do step "$s"; done
