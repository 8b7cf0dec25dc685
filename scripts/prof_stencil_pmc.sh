#!/bin/bash
# PMC counters of the fused stencil kernels (one rocprofv3 pass per counter group, kernel-trace only).
# usage: scripts/prof_stencil_pmc.sh <outdir> [fuse ...]
out=${1:-gpurun_out/stencil_pmc}; shift
mkdir -p "$out"
export TMPDIR=/tmp
for f in ${@:-4}; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
             "SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d "$out/f$f-$i" -o p -- \
      python3 -m parallel_c_programs_amd.cli.run_stencil --steps 4 --warmup 1 --no-check --set fuse=$f > "$out/f$f-$i.log" 2>&1 || exit $?
  done
done
