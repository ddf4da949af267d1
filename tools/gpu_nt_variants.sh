#!/bin/bash
# Nontemporal-store variants: kernel parity tests of this build, then step A/B pairs of this build
# against exp_so/liblcclip_NT_{F32,ATT,LN}.so (f32 epilogue outputs / attention outputs /
# LayerNorm outputs also nontemporal).
source gpu_step.sh
run t_kern 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py
for r in 1 2; do
  run sprod$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  for v in NT_F32 NT_ATT NT_LN; do
    LCCLIP_LIB=exp_so/liblcclip_$v.so run s${v}_$r 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
  done
done
run sprod3 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
