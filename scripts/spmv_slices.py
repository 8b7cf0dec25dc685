"""SpMV lab: time the XCD-sliced kernel with all slices, then one slice at a time (others given no items),
to see which slices (hot narrow ones or wide cold ones) bound the launch. Usage: python scripts/spmv_slices.py [S [head]]"""
import sys

import torch

sys.path.insert(0, ".")
from parallel_c_programs_amd._native import ops as native  # noqa: E402
from parallel_c_programs_amd.parallel.spmv import DistributedSpMV  # noqa: E402
from parallel_c_programs_amd.parallel import init  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 16
HEAD = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0625
ITEM = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
ctx = init(None, None)
d = DistributedSpMV.powerlaw(ctx, 10_000_000, 100_000_000, 2.5, slices=S, head=HEAD, item_nnz=ITEM)
s = d.parts[0][2]  # one rank, one chunk: the whole matrix
x = torch.rand(s.n_cols, device="cuda")


MODE = 0


def bench(meta, reps=20):
    for _ in range(3):
        native().spmv_sliced(s.lrow, s.col, s.val, x, s.items, s.row_mask, s.chunk_base, s.fix, meta, s.ypart, s.extra,
                             s.n_rows, None, MODE | s.mode)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        native().spmv_sliced(s.lrow, s.col, s.val, x, s.items, s.row_mask, s.chunk_base, s.fix, meta, s.ypart, s.extra,
                             s.n_rows, None, MODE | s.mode)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for mode, what in [(1 | 2 << 8, "no x gathers"), (1 << 8, "1 block/CU"), (2 << 8, "2 blocks/CU"),
                   (3 << 8, "3 blocks/CU"), (4 << 8, "4 blocks/CU"), (5 << 8, "5 blocks/CU"), (6 << 8, "6 blocks/CU"),
                   (1 | 5 << 8, "no x gathers, 5 blocks/CU"), (4 | 2 << 8, "LDS row sums, 2 blocks/CU"),
                   (4 | 5 << 8, "LDS row sums, 5 blocks/CU")]:
    MODE = mode
    print(f"mode {mode} ({what}): {bench(s.meta):.3f} ms")
MODE = 0
full = bench(s.meta)
if "--no-slices" in sys.argv:
    print(f"S={S} head={HEAD} item_nnz={ITEM} all slices: {full:.3f} ms  compact partials {s.partials}")
    sys.exit(0)
print(f"S={S} head={HEAD} H={s.head_cols} all slices: {full:.3f} ms  compact partials {s.partials} "
      f"({s.partials / (S * s.n_rows):.1%} of S x rows)  bounds={s.bounds.tolist()}")
nz0, item0 = s.meta[:S], s.meta[S:2 * S + 1]  # meta = [nz0 | item0 | out0]
for k in range(S):
    m = s.meta.clone()
    it = m[S:2 * S + 1]
    keep0, keep1 = int(item0[k]), int(item0[k + 1])
    for j in range(S + 1):  # every other slice: empty item range
        it[j] = keep0 if j <= k else keep1
    nnz_k = int(s.meta[k + 1] - s.meta[k]) if k + 1 < S else s.nnz - int(s.meta[k])
    print(f"slice {k:2d}: {bench(m):.3f} ms  nnz {nnz_k/1e6:.2f}M  items {keep1-keep0}")
