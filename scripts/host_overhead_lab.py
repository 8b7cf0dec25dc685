"""Host-overhead lab: is one rank's distributed step launch-bound at N = 8? On one GPU:

  * stencil: StencilSlab.step on an emulated rank of N=8 (2048-row slab), halo exchange replaced by nothing:
    host issue time per step (no sync) vs device time per step (synced), per fused depth;
  * spmv: the local half of DistributedSpMV.step_padded on an emulated N=8 rank (products + send packing);
  * RCCL p2p host cost: a world-1 NCCL process group sending to / receiving from itself with
    batch_isend_irecv (the call shape of the halo and ghost exchanges), per op count.

If the host issue time per step approaches the device time, the step is launch-bound and the N=8 number is set
by Python + launch overhead, not by the GPU. Run: python scripts/host_overhead_lab.py
"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd.parallel.dist import Context  # noqa: E402
from parallel_c_programs_amd.parallel.spmv import DistributedSpMV  # noqa: E402
from parallel_c_programs_amd.parallel.stencil import StencilSlab  # noqa: E402


class Emulated(Context):
    @property
    def distributed(self):
        return True


def issue_and_device(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / reps * 1e6, (t2 - t0) / reps * 1e6


def main():
    dev = torch.device("cuda", 0)
    for fuse in (4, 6, 8):
        s = StencilSlab(Emulated(rank=3, world=8, device=dev), 16384, 16384, fuse=fuse)
        s._post_exchange = lambda: []
        host, wall = issue_and_device(lambda: s.step(overlap=True))
        print(f"stencil N=8 rank slab fuse={fuse}: host issue {host:6.1f} us/step, wall {wall:6.1f} us/step", flush=True)
        del s
    torch.cuda.empty_cache()

    d = DistributedSpMV.powerlaw(Context(rank=3, world=8, device=dev), 10_000_000, 100_000_000, slices=16)
    xp = torch.rand(d.n_pad, device=dev)
    out = torch.empty_like(xp)
    idx = torch.randint(0, d.rows, (d.n_ghost,), device=dev)  # a send list of the ghost volume's size
    sendbuf = torch.empty(idx.numel(), device=dev)

    def spmv_local():
        W = d.ctx.world
        for c, (a, b, part) in enumerate(d.parts):
            s0 = d.seg[c * W + d.ctx.rank]
            d._mul(part, xp, out[s0:s0 + (b - a)])
            torch.index_select(out, 0, idx[c::d.chunks], out=sendbuf[:idx[c::d.chunks].numel()])

    host, wall = issue_and_device(spmv_local, reps=50)
    print(f"spmv N=8 rank (chunks {d.chunks}): host issue {host:6.1f} us/step, wall {wall:6.1f} us/step", flush=True)
    del d, xp, out
    torch.cuda.empty_cache()

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29555")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    buf = torch.zeros(2, 8 << 20, device=dev)
    for nops in (2, 4, 14):
        def p2p():
            ops = []
            for i in range(nops // 2):
                ops.append(dist.P2POp(dist.isend, buf[0, i * 1024:(i + 1) * 1024], 0))
                ops.append(dist.P2POp(dist.irecv, buf[1, i * 1024:(i + 1) * 1024], 0))
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        host, wall = issue_and_device(p2p, reps=100)
        print(f"rccl batch_isend_irecv {nops:2d} ops (4 KiB each, self): host {host:6.1f} us/call, wall {wall:6.1f} us/call",
              flush=True)
    for n_el in (1024, 1 << 20):
        src, dst = buf[0, :n_el], buf[1, :n_el]
        host, wall = issue_and_device(lambda: dist.all_to_all_single(dst, src), reps=100)
        print(f"rccl all_to_all_single ({n_el * 4 >> 10} KiB, self): host {host:6.1f} us/call, wall {wall:6.1f} us/call",
              flush=True)
        host, wall = issue_and_device(lambda: dist.all_to_all([dst], [src]), reps=100)
        print(f"rccl all_to_all list ({n_el * 4 >> 10} KiB, self): host {host:6.1f} us/call, wall {wall:6.1f} us/call",
              flush=True)
        host, wall = issue_and_device(lambda: dist.all_gather_into_tensor(dst, src), reps=100)
        print(f"rccl all_gather_into_tensor ({n_el * 4 >> 10} KiB): host {host:6.1f} us/call, wall {wall:6.1f} us/call",
              flush=True)
        host, wall = issue_and_device(lambda: dist.all_gather_into_tensor(dst, src, async_op=True).wait(), reps=100)
        print(f"rccl all_gather_into_tensor async+wait ({n_el * 4 >> 10} KiB): host {host:6.1f} us/call, "
              f"wall {wall:6.1f} us/call", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
