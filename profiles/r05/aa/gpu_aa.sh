#!/bin/bash
# r5 evidence pass after the LoRA / prompt-tower half residual stream (tools/r4/gpu_evidence.sh,
# TAG=r05aa): full GPU suite, smoke, the bench lines DESIGN cites, kernel trace, PMC traffic,
# MFMA busy.
TAG=r05aa bash tools/r4/gpu_evidence.sh
