#!/bin/bash
# Two rocprofv3 PMC passes (kernel trace + counters only, never combined with other tracing) over every
# north-star workload, then a per-kernel markdown summary (scripts/pmc_table.py).
# usage: scripts/prof_pmc_all.sh <outdir> [workload ...]
out=${1:-gpurun_out/pmc_all}; shift
ws=${@:-"sgemm reduce scan stencil spmv region3d raycast histeq"}
mkdir -p "$out"
export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
B="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
for w in $ws; do
  for p in A B; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc ${!p} -d "$out/$w-$p" -o p -- \
      python3 -m parallel_c_programs_amd.cli.run_workload "$w" --steps 3 --warmup 1 --no-check > "$out/$w-$p.log" 2>&1 || exit $?
  done
  python3 scripts/pmc_table.py "$out/$w-A" "$out/$w-B" > "$out/$w.md" || exit $?
  echo "== $w"; cat "$out/$w.md"
done
