#!/bin/bash
# r5 evidence pass on the committed code (tools/r4/gpu_evidence.sh with TAG=r05): GPU tests,
# smoke, the bench lines DESIGN cites, kernel trace, PMC traffic, MFMA busy.
TAG=r05 bash tools/r4/gpu_evidence.sh
