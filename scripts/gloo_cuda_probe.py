"""Probe: which torch.distributed ops does the gloo backend accept on CUDA tensors (two processes, one GPU)?
If the exchanges the bench uses all work, the whole N>1 bench path can run on ONE GPU with gloo carrying the
messages (tests/test_gpu_multi.py). Run: python scripts/gloo_cuda_probe.py"""
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    dev = torch.device("cuda", 0)
    res = {}

    def probe(name, fn):
        try:
            fn()
            torch.cuda.synchronize()
            res[name] = "ok"
        except Exception as e:  # noqa: BLE001
            res[name] = f"FAIL {type(e).__name__}: {str(e)[:80]}"

    t = torch.ones(8, device=dev) * (rank + 1)
    probe("all_reduce", lambda: dist.all_reduce(t))
    probe("all_gather_into_tensor", lambda: dist.all_gather_into_tensor(torch.empty(16, device=dev), t))
    probe("all_gather", lambda: dist.all_gather([torch.empty(8, device=dev) for _ in range(2)], t))
    probe("all_to_all_single", lambda: dist.all_to_all_single(torch.empty(8, device=dev), t, [4, 4], [4, 4]))
    probe("broadcast", lambda: dist.broadcast(t, 0))
    probe("batch_isend_irecv", lambda: [w.wait() for w in dist.batch_isend_irecv(
        [dist.P2POp(dist.isend, t, 1 - rank), dist.P2POp(dist.irecv, torch.empty(8, device=dev), 1 - rank)])])
    probe("barrier", lambda: dist.barrier())
    if rank == 0:
        for k, v in res.items():
            print(f"gloo + cuda tensors: {k:24s} {v}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(run, args=(29631,), nprocs=2, join=True)
