source gpu_step.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_mfma
run mfma 200 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof_mfma/pmc -o p -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline
python tools/pmc_mfma_step.py gpurun_out/prof_mfma/pmc gpurun_out/mfma_busy.json > gpurun_out/mfma_busy.txt 2>&1
echo done
