#!/bin/bash
# PMC pass (kernel trace + counters only) over the SpMV combine A/B (scripts/spmv_combine_ab.py 24): instruction mix
# and wave cycles of spmv_combine_kernel (ballot ranks) vs spmv_combine_scan_kernel (byte-packed scan).
# Summaries: python scripts/pmc_summary.py gpurun_out/cbpmc/A/p_counter_collection.csv spmv_combine_kernel (etc.)
export TMPDIR=/tmp
mkdir -p gpurun_out/cbpmc
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $A -d gpurun_out/cbpmc/A -o p -- python3 scripts/spmv_combine_ab.py 24 > gpurun_out/cbpmc/A.log 2>&1 || exit $?
