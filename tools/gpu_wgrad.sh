source gpu_step.sh
run wg_a 60 python -u tools/bench_wgrad.py
M=25216 run wg_b 60 python -u tools/bench_wgrad.py
M=12608 run wg_c 60 python -u tools/bench_wgrad.py
LCLIB=exp_so/noatomic.so run wg_d 60 python -u tools/bench_wgrad.py
LCLIB=exp_so/noatomic.so M=12608 run wg_e 60 python -u tools/bench_wgrad.py
echo done
