"""SpMV 1e8-nnz power-law (the bench section, one GPU): temporal (production) vs non-temporal stores of the sliced
product's compact partials (mode bit 26 of the sliced launch, an explicit per-call parameter). The partials (~340 MB)
are re-read by the combine right after the product; temporal stores may leave part of them in L2 / the 256 MiB MALL.
Same products bit for bit; prints ms per step.
usage: python scripts/spmv_store_lab.py [steps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd.models import workloads as W  # noqa: E402
from parallel_c_programs_amd.parallel import init  # noqa: E402
from parallel_c_programs_amd.utils.harness import timed  # noqa: E402

NT_PARTIALS = 1 << 26
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = init()
sp = W.SpMV(ctx)
(_, _, part), = sp.d.parts  # one rank, one chunk: the sliced product of the whole matrix
y = torch.empty(part.n_rows, device=ctx.device)
outs = {}
for rnd in range(2):
    for ts in (0, 1):
        mode = 0 if ts else NT_PARTIALS
        t = timed(ctx, lambda: part.spmv(sp.xp, y, mode=mode), steps, 3)
        outs[ts] = y.clone()
        print(f"temporal_partials={ts} {1e3 * t / steps:.4f} ms/step {2 * sp.d.local_nnz * steps / t / 1e9:.1f} GFLOP/s",
              flush=True)
print("bit-identical:", torch.equal(outs[0], outs[1]), flush=True)
