"""North-star stencil CLI: 5-point bf16 stencil on an N x N grid (default 16384), row slabs over the ranks with the
halo exchange overlapped with the interior update (GLUP/s). Ancestor: the 4-neighbour update + 1-cell halo of
ref 2-mpi-region-growing/region.c:250-353, promoted to a numeric stencil.

    run_stencil [N] [--fuse T] [--no-overlap] [--graph-steps G] [--per-rank] [--steps S --warmup W] [--no-check]

  --fuse T         updates fused per kernel / halo depth (2, 3, 4, 6, 8; default by slab height: 8 / 8 / 6 / 6 at
                   N = 1 / 2 / 4 / 8 ranks on 16384 rows)
  --no-overlap     exchange the halo, then update every row in one launch (no interior / edge split)
  --graph-steps G  single rank: replay a captured HIP graph of 2 fused launches for the timed steps
  --per-rank       weak scaling: an N x N grid PER rank instead of one N x N grid split over the ranks

Multi-GPU: torchrun --nproc-per-node 8 -m parallel_c_programs_amd.cli.run_stencil. The check compares a small
grid through the same distributed path bit for bit with the single-domain oracle."""
from .run_workload import run


def _args(ap):
    ap.add_argument("n", nargs="?", type=int, default=16384)
    ap.add_argument("--fuse", type=int, default=0)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--graph-steps", type=int, default=0)
    ap.add_argument("--per-rank", action="store_true")


def _cfg(a):
    return {"n": a.n, "fuse": a.fuse, "overlap": not a.no_overlap, "graph_steps": a.graph_steps,
            "per_rank": a.per_rank}


def main(argv=None) -> int:
    run("stencil", argv, {"n": 16384}, _args, _cfg, doc=__doc__, time_line=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
