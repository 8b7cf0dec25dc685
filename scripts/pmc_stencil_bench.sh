#!/bin/bash
# PMC passes over the bench-config stencil (16384^2 bf16, T = 8 fused levels per launch; run_stencil, one rank),
# kernel trace + counters only, one rocprofv3 run per counter group; per-kernel averages per dispatch in
# $out/summary.txt. Group 3 (matrix-core counters) runs last: a counter name this rocprofv3 does not know ends the
# script there, after the other groups have been written.
out=${1:-gpurun_out/stencil_bench_pmc}
fuse=${2:-8}
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_COUNT TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d "$out/p$i" -o p -- \
    python3 -m parallel_c_programs_amd.cli.run_stencil --fuse "$fuse" --steps 6 --warmup 2 --no-check \
    > "$out/p$i.log" 2>&1 || { echo "pass $i failed (rc $?)"; break; }
done
python3 - "$out" <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "stencil" not in k:
            continue
        name = k.replace("(anonymous namespace)::", "").split("(")[0]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(f"{out}/summary.txt", "w") as fo:
    for name, cs in sorted(agg.items()):
        fo.write(f"== {name}\n")
        for c, v in sorted(cs.items()):
            fo.write(f"  {c:28s} {sum(v) / len(v):.4g}   (n={len(v)})\n")
print(open(f"{out}/summary.txt").read())
PY
