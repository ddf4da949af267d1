source gpu_step.sh
run tk 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "every_tile"
TILES=0,4,8,9,10,1 run sk 120 python -u tools/bench_skinny.py
echo done
