"""One window of a rocprofv3 --hip-trace --kernel-trace database as a single chronological listing: the host API calls
(thread, start, duration) and the device kernels (stream, start, duration), relative to the start of one kernel.
Used to see what a library enqueues around a call (round 6: what RCCL adds per grouped send / recv).
Run: python scripts/rocpd_api_window.py <results.db> <kernel-substring> [which=-5] [before_us=250] [after_us=120]"""
import sqlite3
import sys


def main():
    db, sub = sys.argv[1], sys.argv[2]
    which = int(sys.argv[3]) if len(sys.argv) > 3 else -5
    before = float(sys.argv[4]) if len(sys.argv) > 4 else 250.0
    after = float(sys.argv[5]) if len(sys.argv) > 5 else 120.0
    c = sqlite3.connect(f"file:{db}?mode=ro", uri=True)  # read-only: a wrong path fails instead of creating a file
    ks = c.execute("select name, start, end, stream_id, corr_id from kernels where name like ? order by start",
                   (f"%{sub}%",)).fetchall()
    if not ks:
        sys.exit(f"no kernel matching {sub!r}")
    name, kstart, kend, kstream, _ = ks[which]
    t0 = kstart  # host and device timestamps share one clock in rocprofv3's database
    lo, hi = t0 - before * 1e3, t0 + after * 1e3
    rows = [("host", r[1], r[2], f"tid {r[3]}", r[0]) for r in c.execute(
        "select name, start, end, tid from regions where start between ? and ? and name not like '__hipRegister%' "
        "order by start", (lo, hi))]
    rows += [("dev", k[1], k[2], f"stream {k[3]}", k[0].split("(")[0][:70]) for k in c.execute(
        "select name, start, end, stream_id from kernels where end >= ? and start <= ? order by start", (lo, hi))]
    print(f"window around launch of {name.split('(')[0][:60]} (#{which}); times in us from that kernel's start")
    for kind, s, e, where, nm in sorted(rows, key=lambda r: r[1]):
        print(f"{kind:4s} {(s - t0) / 1e3:9.2f} +{(e - s) / 1e3:8.2f}  {where:12s} {nm}")


if __name__ == "__main__":
    main()
