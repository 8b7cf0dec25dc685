"""Exchange windows of the N = 8 SpMV rank step from a rocprofv3 kernel trace of scripts/spmv_host_lab.py with
SPMV_LAB_RCCL=1 (round 6): per step, when each exchange's RCCL kernel started and how long it could run before the
compute stream needs its data in a stall-free schedule, and the exposure of an xGMI transfer of the real byte counts at
several inbound bandwidths (no GPU needed).

  ex0 (chunk 0, posted after its combine): needed by the next step's paired phase-0 launch, which in a stall-free
      schedule starts when chunk 1's combine ends -> W0 = comb1.end - rccl0.start
  ex1 (chunk 1, posted at the end of the step): needed by the next step's chunk-0 phase-1 launch, which starts when
      the paired phase-0 launch ends -> W1 = P0(next).end - rccl1.start
usage: python scripts/spmv_windows.py <results.db> [bytes0,bytes1] [latency_us]"""
import sqlite3
import statistics
import sys


def main():
    db = sys.argv[1]
    nb = [float(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [10603376.0, 10070956.0]
    lat = float(sys.argv[3]) if len(sys.argv) > 3 else 5.0
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels where name like '%spmv%' or name like '%rccl%' "
                     "order by start").fetchall()
    ev = []
    for name, s, e in rows:
        if "rccl" in name:
            kind = "X"
        elif "combine" in name:
            kind = "C"
        elif "true, true" in name:  # the paired phase-0 launch
            kind = "P0"
        else:
            kind = "P1"
        ev.append((kind, s / 1e3, e / 1e3))
    # steps: P0, P1, C, P1, C with X's interleaved; walk the compute kernels in order
    comp = [x for x in ev if x[0] != "X"]
    xs = [x for x in ev if x[0] == "X"]
    w0, w1, d0, d1, steps = [], [], [], [], []
    i = 0
    while i + 5 < len(comp):
        if comp[i][0] != "P0" or [k for k, _, _ in comp[i:i + 6]] != ["P0", "P1", "C", "P1", "C", "P0"]:
            i += 1
            continue
        p0, p1a, c0, p1b, c1, p0n = comp[i:i + 6]
        x0 = next((x for x in xs if x[1] >= c0[2] - 1 and x[1] < c1[2] + 20), None)
        x1 = next((x for x in xs if x[1] >= c1[2] - 1 and x[1] < p0n[2]), None)
        if x0 and x1:
            w0.append(c1[2] - x0[1]), w1.append(p0n[2] - x1[1])
            d0.append(x0[2] - x0[1]), d1.append(x1[2] - x1[1])
            steps.append(p0n[1] - p0[1])
        i += 5
    med = statistics.median
    print(f"steps analysed: {len(steps)}; step (P0 start to next P0 start) median {med(steps):.1f} us")
    print(f"ex0: window W0 median {med(w0):.1f} us (min {min(w0):.1f}); local RCCL kernel {med(d0):.1f} us")
    print(f"ex1: window W1 median {med(w1):.1f} us (min {min(w1):.1f}); local RCCL kernel {med(d1):.1f} us")
    print(f"exposure of an xGMI transfer of {nb[0] / 1e6:.2f} / {nb[1] / 1e6:.2f} MB (+ {lat:.0f} us start-up) per "
          f"exchange, against the median windows:")
    print(f"{'inbound GB/s':>12s} {'T0 us':>7s} {'T1 us':>7s} {'exposed0':>9s} {'exposed1':>9s} {'total':>7s}")
    for bw in (300, 450, 600, 800):
        t0, t1 = nb[0] / (bw * 1e3) + lat, nb[1] / (bw * 1e3) + lat
        e0, e1 = max(0.0, t0 - med(w0)), max(0.0, t1 - med(w1))
        print(f"{bw:12d} {t0:7.1f} {t1:7.1f} {e0:9.1f} {e1:9.1f} {e0 + e1:7.1f}")


if __name__ == "__main__":
    main()
