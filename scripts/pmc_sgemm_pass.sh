set -e
export TMPDIR=/tmp
for v in 16 7; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_LDS -d gpurun_out/sgpmc_$v -o p -- python3 scripts/sgemm_pmc.py 8192 $v > gpurun_out/sgpmc_$v.log 2>&1
done
