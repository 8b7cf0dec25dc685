"""Per-kernel PMC summary of one workload from two rocprofv3 passes (scripts/prof_pmc_all.sh):
python scripts/pmc_table.py <passA dir> <passB dir>. Values are means per dispatch; counters are summed over
the 8 XCDs by rocprofv3 (GRBM_GUI_ACTIVE too, so it is divided by 8 for the per-die cycle count)."""
import collections
import csv
import glob
import sys


def load(d):
    agg, n, dur = collections.defaultdict(float), collections.Counter(), collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: agg[k] / n[k] for k in agg}, dur


def short(name):
    for p in ("void ", "(anonymous namespace)::"):
        name = name.replace(p, "")
    return name.split("(")[0][:56]


a, dur = load(sys.argv[1])
b, _ = load(sys.argv[2])
kernels = sorted({k for k, _ in a} | {k for k, _ in b}, key=lambda k: -sum(dur.get(k, [0])))
print("| kernel | calls | µs/call | waves | VALU/wave | VMEM rd+wr/wave | LDS/wave | LDS bank confl. | MFMA f32 util | L2 hit | fabric req GB/s (64 B/req) |")
print("|---|---|---|---|---|---|---|---|---|---|---|")
for k in kernels:
    g = lambda c, src=a: src.get((k, c))  # noqa: E731
    us = sum(dur.get(k, [0])) / max(1, len(dur.get(k, [])))
    waves = g("SQ_WAVES") or 0
    per = lambda c: f"{g(c) / waves:.0f}" if waves and g(c) is not None else "-"  # noqa: E731
    vmem = f"{((g('SQ_INSTS_VMEM_RD') or 0) + (g('SQ_INSTS_VMEM_WR') or 0)) / waves:.0f}" if waves and g("SQ_INSTS_VMEM_RD") is not None else "-"
    cyc = (g("GRBM_GUI_ACTIVE") or 0) / 8
    # MFMA_MOPS_F32: units of 512 FLOP per count (rocprof derived-metric convention) vs 256 CUs x 256 FLOP/clk f32
    mops = g("SQ_INSTS_VALU_MFMA_MOPS_F32")
    util = f"{100 * mops * 512 / (cyc * 256 * 256):.0f}%" if mops and cyc else "-"
    hit, miss = g("TCC_HIT_sum", b), g("TCC_MISS_sum", b)
    l2 = f"{100 * hit / (hit + miss):.0f}%" if hit is not None and hit + miss > 0 else "-"
    rd, wr = g("TCC_EA0_RDREQ_sum", b), g("TCC_EA0_WRREQ_sum", b)
    hbm = f"{(rd + wr) * 64 / (us * 1e-6) / 1e9:.0f}" if rd is not None and wr is not None and us > 0 else "-"
    conf = f"{g('SQ_LDS_BANK_CONFLICT'):.3g}" if g("SQ_LDS_BANK_CONFLICT") is not None else "-"
    print(f"| {short(k)} | {len(dur.get(k, []))} | {us:.1f} | {waves:.0f} | {per('SQ_INSTS_VALU')} | {vmem} | "
          f"{per('SQ_INSTS_LDS')} | {conf} | {util} | {l2} | {hbm} |")
