source gpu_step.sh
run prange 60 python -c "import torch; print('priority_range', torch.cuda.Stream.priority_range())"
run b00 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
LCCLIP_GRAD_PRIO=1 LCCLIP_TEXT_PRIO=1 run b11 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
LCCLIP_GRAD_PRIO=1 run b10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
LCCLIP_TEXT_PRIO=-1 run b01 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
run b00b 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
