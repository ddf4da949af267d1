source gpu_step.sh
TILES=0,9,10,0 run sk 120 python -u tools/bench_skinny.py
echo done
