#!/bin/bash
# PMC passes for one GEMM shape per variant (run on the GPU box). Args: tag; env N K EPI.
set -e
export TMPDIR=/tmp
for V in ${VS:-1 6}; do
  export V
  timeout -k 10 120 python tools/gemm_one.py
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA --output-format csv -d gpurun_out/pmc_$1_v${V}_a -o p -- python tools/gemm_one.py > /dev/null 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_$1_v${V}_b -o p -- python tools/gemm_one.py > /dev/null 2>&1
done
