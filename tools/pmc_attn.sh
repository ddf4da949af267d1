#!/bin/bash
# PMC passes over tools/bench_attn.py (run on the GPU box, from the repo root). FETCH_SIZE (3 TCC
# slots) and WRITE_SIZE (2) never share a pass (4 TCC slots per pass).
set -e
export TMPDIR=/tmp REPS=3 FORMS=${FORMS:-0}
P=gpurun_out/pmc_attn
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d ${P}_a -o p -- python tools/bench_attn.py > /dev/null 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE FETCH_SIZE --output-format csv -d ${P}_b -o p -- python tools/bench_attn.py > /dev/null 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS WRITE_SIZE --output-format csv -d ${P}_c -o p -- python tools/bench_attn.py > /dev/null 2>&1
python tools/pmc_report.py attn ${P}_a ${P}_b ${P}_c > gpurun_out/pmc_attn_report.txt 2>&1
echo done
