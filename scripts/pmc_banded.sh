#!/bin/bash
# PMC passes (kernel trace + counters only, one rocprofv3 run per counter group) over the banded SpMV lab at the
# reference config: variant 1 (row per wave, 4-B loads) and variant 8 (block stream, 16-B loads); per-kernel
# averages in $out/summary.txt.
out=${1:-gpurun_out/banded_pmc}
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d "$out/p$i" -o p -- \
    python3 scripts/spmv_banded_lab.py 100000 401 200 100 200 10 1,8 > "$out/p$i.log" 2>&1 || exit $?
done
python3 - "$out" <<'PY'
import collections, csv, glob, sys
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "banded" not in k:
            continue
        name = k.replace("(anonymous namespace)::", "").split("(")[0][-70:]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(f"{out}/summary.txt", "w") as fo:
    for name, cs in sorted(agg.items()):
        fo.write(f"== {name}\n")
        for c, v in sorted(cs.items()):
            fo.write(f"  {c:26s} {sum(v) / len(v):.4g}\n")
print(open(f"{out}/summary.txt").read())
PY
