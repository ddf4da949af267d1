#!/bin/bash
# r5: what the side streams buy at B = 256 (same box, interleaved): text tower and PEFT weight
# gradients on side streams (default) vs on the main stream; and the HIP-graph replay.
source gpu_step.sh
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  run m_default_$i 300 $B
  LCCLIP_OVERLAP_TEXT=0 run m_notext_$i 300 $B
  LCCLIP_OVERLAP_GRADS=0 run m_nograds_$i 300 $B
  run m_graph_$i 300 $B --graph
done
grep -Ho '"value": [0-9.]*' gpurun_out/m_*.log
