#!/bin/bash
# Memory-pipeline counters of the production SpMV (TA / TCP / TCC busy and stall cycles), kernel trace only.
export TMPDIR=/tmp
out=${1:-gpurun_out/spmv_ta}
mkdir -p $out
i=0
for grp in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCC_TAG_STALL_sum TCC_BUSY_sum TCC_REQ_sum GRBM_GUI_ACTIVE" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_TOTAL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_IB_STALL_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $out/p$i -o p -- \
    python3 bench.py --sections spmv --steps 5 --warmup 1 --no-ref > $out/p$i.log 2>&1 || exit $?
done
for k in spmv_sliced spmv_combine; do for f in $out/p*/p_counter_collection.csv; do echo "== $k $f"; python3 scripts/pmc_summary.py $f $k; done; done
