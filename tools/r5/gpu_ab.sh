#!/bin/bash
# r5 final evidence pass (tools/r4/gpu_evidence.sh, TAG=r05ab): full GPU suite, smoke, the bench
# lines DESIGN cites, kernel trace, PMC traffic, MFMA busy — on the round's final code.
TAG=r05ab bash tools/r4/gpu_evidence.sh
