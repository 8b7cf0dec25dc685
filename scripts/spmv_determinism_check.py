import sys, torch
sys.path.insert(0, '.')
from parallel_c_programs_amd.parallel.dist import Context
from parallel_c_programs_amd.parallel.spmv import DistributedSpMV
dev = torch.device("cuda", 0)
d = DistributedSpMV.powerlaw(Context(device=dev), 10_000_000, 100_000_000, slices=16)
part = d.parts[0][2]
x = torch.rand(d.n_pad, device=dev)
a = part.spmv(x).clone(); b = part.spmv(x).clone(); c = part.spmv(x).clone()
print("fix entries", part.fix.shape[0], "identical", torch.equal(a, b), torch.equal(a, c), flush=True)
