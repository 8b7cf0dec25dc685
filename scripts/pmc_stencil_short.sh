#!/bin/bash
# PMC passes over the short-slab stencil sweep (bin/stencil_lab, STENCIL_ROWS=2048, STENCIL_SWEEP=short), kernel
# trace + counters only, one pass per counter group; summary per kernel instance in $out/summary.txt.
out=${1:-gpurun_out/stencil_short_pmc}; shift
mkdir -p "$out"
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include -Icsrc/kernels -Icsrc/runtime scripts/stencil_lab.hip \
  -o /tmp/stencil_lab 2>/dev/null || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  STENCIL_ROWS=2048 STENCIL_SWEEP=short timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp \
    -d "$out/p$i" -o p -- /tmp/stencil_lab ${@:-4 6} > "$out/p$i.log" 2>&1 || exit $?
done
python3 - "$out" <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "stencil5xT2" not in k:
            continue
        name = k.split("stencil5xT2_kernel<")[1].split(">")[0] if "<" in k else k[:80]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(f"{out}/summary.txt", "w") as fo:
    for name, cs in sorted(agg.items()):
        fo.write(f"== stencil5xT2_kernel<{name}>\n")
        for c, v in sorted(cs.items()):
            fo.write(f"  {c:26s} {sum(v) / len(v):.4g}\n")
print(open(f"{out}/summary.txt").read())
PY
