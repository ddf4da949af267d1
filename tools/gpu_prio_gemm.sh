source gpu_step.sh
# ping-pong GEMM compute-segment priority sweep (exp_so/pr<N>.so built with -DLC_PP_PRIO=N)
VARIANTS=5 run base 200 python -u tools/bench_gemm.py
for pr in 0 2 3; do LCLIB=exp_so/pr$pr.so VARIANTS=5 run pr$pr 200 python -u tools/bench_gemm.py; done
VARIANTS=5 run base2 200 python -u tools/bench_gemm.py
echo done
