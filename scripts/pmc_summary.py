"""Average PMC counters per dispatch of the kernels matching a substring: python scripts/pmc_summary.py <csv> <substr>"""
import collections
import csv
import sys

agg, n = collections.defaultdict(float), collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
for k in sorted(agg):
    print(f"{k:28s} {agg[k] / n[k]:.4g}")
