"""Summarise a rocprofv3 rocpd database (default output of `rocprofv3 --kernel-trace`) without a GPU:
dispatches of the same kernel + grid size are folded into one row (first-seen order; calls, mean / min us).

usage: python scripts/rocpd_runs.py <results.db> [name-substring]
"""
import sqlite3
import sys


def main():
    db, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    c = sqlite3.connect(f"file:{db}?mode=ro", uri=True)  # read-only: a wrong path fails instead of creating a file
    rows = c.execute("select name, grid_x, workgroup_x, duration from kernels order by start").fetchall()
    runs, index = [], {}
    for name, gx, wx, dur in rows:
        if sub and sub not in name:
            continue
        key = (name.replace("(anonymous namespace)::", "").split("(")[0], gx // max(wx, 1))
        if key in index:
            runs[index[key]][1].append(dur)
        else:
            index[key] = len(runs)
            runs.append((key, [dur]))
    print(f"{'kernel':60s} {'blocks':>7s} {'calls':>6s} {'mean us':>9s} {'min us':>8s}")
    for (name, blocks), d in runs:
        print(f"{name[:60]:60s} {blocks:7d} {len(d):6d} {sum(d) / len(d) / 1e3:9.2f} {min(d) / 1e3:8.2f}")


if __name__ == "__main__":
    main()
