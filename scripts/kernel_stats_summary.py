"""Summarises a rocprofv3 `--stats --output-format csv` kernel_stats.csv as a markdown table (top kernels by total
time, demangled names shortened): python scripts/kernel_stats_summary.py gpurun_out/prof/b_kernel_stats.csv [top]"""
import csv
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    cut = name.find("(")
    return (name[:cut] if cut > 0 else name)[:90]


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {path}: {len(rows)} kernels, {total / 1e6:.1f} ms of kernel time in total\n")
    print("| kernel | calls | total ms | mean us | min us | max us | share |")
    print("|---|---|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {t / 1e6:.2f} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"{float(r['MinNs']) / 1e3:.1f} | {float(r['MaxNs']) / 1e3:.1f} | {100 * t / total:.1f}% |")


if __name__ == "__main__":
    main()
