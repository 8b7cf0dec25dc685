"""Print the dispatch timeline (start offset, duration, stream, kernel) of the last N kernels of a rocprofv3 rocpd
database whose name matches any of the given substrings, relative to the first printed one (no GPU needed).

usage: python scripts/rocpd_timeline.py <results.db> <count> [substr,substr,...]
"""
import sqlite3
import sys


def main():
    db, count = sys.argv[1], int(sys.argv[2])
    subs = sys.argv[3].split(",") if len(sys.argv) > 3 else [""]
    c = sqlite3.connect(f"file:{db}?mode=ro", uri=True)  # read-only: a wrong path fails instead of creating a file
    rows = c.execute("select name, start, end, stream_id, queue_id, grid_x / max(workgroup_x, 1) "
                     "from kernels order by start").fetchall()
    rows = [r for r in rows if any(s in r[0] for s in subs)][-count:]
    t0 = rows[0][1]
    print(f"{'start us':>9s} {'end us':>9s} {'dur us':>8s} {'stream':>6s} {'queue':>5s} {'blocks':>7s}  kernel")
    for name, s, e, st, q, blocks in rows:
        nm = name.replace("(anonymous namespace)::", "").split("(")[0]
        print(f"{(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f} {st:6d} {q:5d} {blocks:7d}  {nm[:90]}")


if __name__ == "__main__":
    main()
