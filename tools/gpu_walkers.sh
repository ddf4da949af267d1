source gpu_step.sh
for i in 1 2; do
for w in 0 64 128; do
  (export LC_TN_WALKERS=$w; run w${w}_$i 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline) || exit $?
done
done
echo done
