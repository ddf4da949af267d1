#!/bin/bash
# r4 evidence pass on the committed code: GPU tests, smoke, bench lines, kernel trace, PMC
# traffic (tools/gpu_round_end.sh) and the MFMA-busy counter pass (tools/gpu_mfma_pmc.sh).
TAG=${TAG:-r04} bash tools/gpu_round_end.sh || exit $?
bash tools/gpu_mfma_pmc.sh
