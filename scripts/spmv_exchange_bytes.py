"""Per-rank exchange bytes of the N-rank SpMV ghost layout on the 1e8-nnz / 1e7-row power-law matrix (round 6): every
rank's send and receive bytes per row chunk, from the REAL send lists (each owner learns which of its rows every peer
references: the same set-up exchange as the GPU job), for a given row chunk 0 fraction. CPU / gloo, no GPU needed.
usage: python scripts/spmv_exchange_bytes.py [world] [frac ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd.parallel.dist import spawn  # noqa: E402
from parallel_c_programs_amd.parallel.spmv import DistributedSpMV  # noqa: E402


def _rank(ctx, fracs, out_dir):
    torch.set_num_threads(1)
    lines = []
    for f in fracs:
        d = DistributedSpMV.powerlaw(ctx, 10_000_000, 100_000_000, chunks=2, colsplit=False, chunk0_frac=f)
        W, r = ctx.world, ctx.rank
        send = [4 * sum(d.send_counts[c][q] for q in range(W) if q != r) for c in range(2)]
        recv = [4 * sum(d.recv_counts[c][q] for q in range(W) if q != r) for c in range(2)]
        per_peer_max = [max(4 * d.send_counts[c][q] for q in range(W) if q != r) for c in range(2)]
        lines.append(f"frac {f:.2f} rank {r}: rows {d.rows} chunk rows {[b - a for a, b in (d.chunk_rows(c) for c in range(2))]} "
                     f"send MB {[round(b / 1e6, 2) for b in send]} recv MB {[round(b / 1e6, 2) for b in recv]} "
                     f"largest single-peer message per chunk MB {[round(b / 1e6, 2) for b in per_peer_max]}")
        del d
    with open(os.path.join(out_dir, f"{ctx.rank}.txt"), "w") as fh:
        fh.write("\n".join(lines) + "\n")


def main():
    import tempfile

    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    fracs = [float(v) for v in sys.argv[2:]] or [0.5, 0.4]
    with tempfile.TemporaryDirectory() as td:
        spawn(_rank, world, "gloo", (fracs, td))
        for r in range(world):
            print(open(os.path.join(td, f"{r}.txt")).read(), end="")


if __name__ == "__main__":
    main()
