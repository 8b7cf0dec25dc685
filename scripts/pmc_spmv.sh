#!/bin/bash
# Two PMC passes (kernel trace + counters only) over the SpMV slice lab: instruction mix and wait/active cycles.
export TMPDIR=/tmp
mkdir -p gpurun_out/sppmc
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
B="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $A -d gpurun_out/sppmc/A -o p -- python3 scripts/spmv_slices.py 16 0.0625 1024 --no-slices > gpurun_out/sppmc/A.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $B -d gpurun_out/sppmc/B -o p -- python3 scripts/spmv_slices.py 16 0.0625 1024 --no-slices > gpurun_out/sppmc/B.log 2>&1 || exit $?
