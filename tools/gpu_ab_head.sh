source gpu_step.sh
# same-box A/B: the committed HEAD vs the working tree. Set up first (and remove afterwards):
#   git worktree add exp_head HEAD && make -C exp_head/lifelong-clip_amd/csrc -j8
run tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread
run adk 100 python -u tools/bench_adapter_kernels.py
for i in 1 2; do
  run head$i 200 python -u exp_head/bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run new$i 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
echo done
