#!/bin/bash
# r5 evidence pass after the half residual stream (tools/r4/gpu_evidence.sh, TAG=r05v): full GPU
# suite, smoke, the bench lines DESIGN cites, kernel trace, PMC traffic, MFMA busy.
TAG=r05v bash tools/r4/gpu_evidence.sh
