source gpu_step.sh
for v in trace NODMA NOREAD; do LCLIB=exp_so/$v.so K=3072 run w4_$v 100 python -u tools/w4_trace.py; done
