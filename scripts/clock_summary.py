"""Per-dispatch GRBM_GUI_ACTIVE / duration of the kernels in a rocprofv3 counter_collection.csv, grouped by kernel:
first / middle / last calls. usage: python scripts/clock_summary.py <counter_collection.csv> [substring ...]"""
import collections
import csv
import sys

rows = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
        continue
    name = r["Kernel_Name"]
    if len(sys.argv) > 2 and not any(s in name for s in sys.argv[2:]):
        continue
    dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows[name[:90]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), dur))
for name, v in rows.items():
    v.sort()
    ratio = [g / d for _, g, d in v if d > 0]
    durs = [d / 1e3 for _, _, d in v]
    k = max(1, len(v) // 4)
    print(f"{name}\n  calls {len(v)}  GRBM/ns first {sum(ratio[:k]) / k:.3f} last {sum(ratio[-k:]) / k:.3f}"
          f"  us first {sum(durs[:k]) / k:.1f} last {sum(durs[-k:]) / k:.1f}")
