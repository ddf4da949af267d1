source gpu_step.sh
# A/B of an env toggle on one box: AB_OFF="VAR=value" for the baseline runs, alternating
for i in 1 2; do
  (export $AB_OFF; run off$i 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline) || exit $?
  run on$i 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
done
echo done
