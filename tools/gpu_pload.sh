source gpu_step.sh
VARIANTS=5 run base 200 python -u tools/bench_gemm.py
for pl in 0 1 3 4; do LCLIB=exp_so/pl$pl.so VARIANTS=5 run pl$pl 200 python -u tools/bench_gemm.py; done
VARIANTS=5 run base2 200 python -u tools/bench_gemm.py
echo done
