#!/bin/bash
source gpu_step.sh
run f_rounds 200 python -u tools/r4/tile_rounds.py
run f_rounds768 200 env K=768 python -u tools/r4/tile_rounds.py
echo done
