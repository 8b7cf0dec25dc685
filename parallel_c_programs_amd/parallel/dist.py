"""Process-group context: one process per GPU over RCCL (torch.distributed backend "nccl" is RCCL on ROCm,
riding xGMI between MI355Xs), or gloo on CPU for GPU-less tests.

Replaces the reference's MPI bootstrap (MPI_Init / Comm_size / Comm_rank / Finalize: 1-introduction/mpi.c:10-44,
2-mpi-region-growing/region.c:537-548). Launch with
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 <script> ...
or, for tests, `spawn(fn, world, backend="gloo")`.
"""
from __future__ import annotations

import os
import socket
from dataclasses import dataclass
from datetime import timedelta

import torch
import torch.distributed as dist


@dataclass
class Context:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def distributed(self) -> bool:
        return self.world > 1 and dist.is_initialized()

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    def barrier(self) -> None:
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.distributed:
            dist.all_reduce(t, op=_OPS[op])
        return t

    def all_reduce_async(self, t: torch.Tensor, op: str = "sum"):
        """In-place all-reduce left in flight: returns the work whose wait() orders the caller's stream after it (None
        when not distributed). Lets a step's collective overlap the next step's compute (Reduce.step)."""
        if not self.distributed:
            return None
        return dist.all_reduce(t, op=_OPS[op], async_op=True)

    def all_gather(self, t: torch.Tensor) -> list[torch.Tensor]:
        if not self.distributed:
            return [t]
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t.contiguous())
        return out

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.distributed:
            dist.broadcast(t, src)
        return t

    def exchange(self, outs: list, ins: list, async_op: bool = False) -> list:
        """The one all-to-all primitive every N > 1 exchange goes through (halo rows, z-slab planes, SpMV ghost
        entries): ins[q] is sent to rank q, outs[q] is received from rank q; zero-size entries (non-neighbours, self)
        move nothing. RCCL: ONE list all_to_all (grouped per-peer sends/receives over the point-to-point xGMI links,
        ~19 us of host time against ~10 us per op for a batch of P2P ops, scripts/host_overhead_lab.py). gloo has
        no list all_to_all: a P2P batch over the non-empty entries, host-staged for CUDA tensors (gloo's P2P ops
        are not stream-ordered: the transport that lets several ranks share one GPU in tests).
        Every rank must call it (collective), also with nothing to send. Returns the works to wait on (empty when
        async_op is False)."""
        if not self.distributed:
            return []
        if len(outs) != self.world or len(ins) != self.world:
            raise ValueError("exchange: one (possibly empty) tensor per rank")
        if self.backend == "nccl":
            w = dist.all_to_all(outs, ins, async_op=True)
        else:
            staged_io = any(t.is_cuda for t in outs + ins)
            ops, staged = [], []
            for q in range(self.world):
                if q == self.rank:
                    if outs[q].numel():
                        outs[q].copy_(ins[q])
                    continue
                if ins[q].numel():
                    ops.append(dist.P2POp(dist.isend, ins[q].cpu() if staged_io else ins[q], q))
                if outs[q].numel():
                    buf = torch.empty(outs[q].shape, dtype=outs[q].dtype) if staged_io else outs[q]
                    ops.append(dist.P2POp(dist.irecv, buf, q))
                    staged.append((outs[q], buf))
            w = dist.batch_isend_irecv(ops) if ops else []
            if staged_io:
                for x in w:
                    x.wait()
                for dst, buf in staged:
                    if buf is not dst:
                        dst.copy_(buf)
                return []
        works = w if isinstance(w, list) else [w]
        if async_op:
            return works
        for x in works:
            x.wait()
        return []

    def exchange_segments(self, slot: int, send: torch.Tensor, soff: list, scnt: list, recv: torch.Tensor, roff: list,
                          rcnt: list) -> list:
        """Asynchronous exchange of contiguous segments: send[soff[q] : soff[q] + scnt[q]] goes to rank q and
        recv[roff[q] : roff[q] + rcnt[q]] is received from rank q (one entry per rank, zero counts move nothing).
        Returns the works to wait on. On RCCL with GPU buffers of one dtype it takes the NATIVE path (NativeExchange: a
        dedicated RCCL communicator driven from C++, ~an order of magnitude less host time than a torch all_to_all;
        `slot` names the exchange in flight, one per concurrently pending exchange); otherwise the same segments
        as views through exchange() (gloo, LazyContext, CPU tensors)."""
        if not self.distributed:
            return []
        nx = native_exchange(self) if send.is_cuda and send.dtype == recv.dtype else None
        if nx is not None:
            return nx.post(slot, send, soff, scnt, recv, roff, rcnt)
        ins = [send[o:o + n] for o, n in zip(soff, scnt)]
        outs = [recv[o:o + n] for o, n in zip(roff, rcnt)]
        return self.exchange(outs, ins, async_op=True)

    def neighbour_exchange(self, pairs, async_op: bool = False) -> list:
        """Sends / receives with a few peers: pairs = [(peer, send tensor, recv tensor)], each peer at most once,
        tensors contiguous (possibly no pairs: the rank still takes part in the collective)."""
        if not self.distributed:
            return []
        peers = [p for p, _, _ in pairs]
        if len(set(peers)) != len(peers):
            raise ValueError(f"neighbour_exchange: peer listed twice in {peers}")
        like = pairs[0][1] if pairs else torch.empty(0, device=self.device)
        empty = like.new_empty(0)
        ins, outs = [empty] * self.world, [empty] * self.world
        for peer, snd, rcv in pairs:
            ins[peer], outs[peer] = snd, rcv
        return self.exchange(outs, ins, async_op)

    def _staged(self, t: torch.Tensor) -> bool:
        """gloo moves CUDA tensors point-to-point without stream ordering: such messages go through host copies."""
        return self.backend == "gloo" and t.is_cuda

    def send(self, t: torch.Tensor, dst: int) -> None:
        dist.send(t.cpu() if self._staged(t) else t.contiguous(), dst)

    def recv(self, t: torch.Tensor, src: int) -> None:
        if self._staged(t):
            buf = torch.empty(t.shape, dtype=t.dtype)
            dist.recv(buf, src)
            t.copy_(buf)
        else:
            dist.recv(t, src)

    def scalar(self, v, dtype=torch.float64) -> torch.Tensor:
        return torch.tensor([v], dtype=dtype, device=self.device)

    def max_over_ranks(self, v: float) -> float:
        t = self.scalar(float(v))
        self.all_reduce_(t, "max")
        return float(t.item())


class _NativeWork:
    def __init__(self, nx, slot):
        self.nx, self.slot = nx, slot

    def wait(self):
        self.nx.C.xcomm_wait(self.nx.handle, self.slot, self.nx.device)


class NativeExchange:
    """A dedicated RCCL communicator for per-step exchanges (csrc/comm/exchange_rccl.hip): rank 0's ncclUniqueId is
    broadcast over the job's process group once, then every exchange is ONE C++ call (grouped ncclSend / ncclRecv per
    peer on the communicator's stream, ordered after the caller's stream by an event) and its wait another (the
    caller's stream waits for the slot's done event). Created on first use by Context.exchange_segments, on every
    rank at the same program point (the exchange calls themselves are collective). PCMX_NATIVE_EXCHANGE=0 turns it
    off (torch all_to_all instead)."""

    def __init__(self, ctx: Context):
        from .. import _C

        self.C, self.device, self.handle = _C, ctx.device.index, 0
        obj = [_C.xcomm_unique_id() if ctx.rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        # proven before first use: one float to / from every peer, host-waited with a timeout (a hung or failed probe
        # aborts the communicator), then agreed over the job's own process group — a failure on ANY rank (creation
        # included) sends every rank to the torch path together, so no rank is left in a collective the others skip
        rc = 0
        try:
            self.handle = _C.xcomm_create(obj[0], ctx.world, ctx.rank, self.device)
        except RuntimeError:
            rc = -1
        if self.handle:
            rc = _C.xcomm_probe(self.handle, int(float(os.environ.get("PCMX_XCOMM_PROBE_S", "60")) * 1000))
        if os.environ.get("PCMX_XCOMM_FAIL_RANK") == str(ctx.rank):  # test hook: this rank reports a failed probe
            rc = rc or -2
        if ctx.max_over_ranks(0.0 if rc == 0 else 1.0) != 0.0:
            self.close()
            raise RuntimeError(f"native exchange unavailable (rank {ctx.rank}: rc {rc})")

    def post(self, slot, send, soff, scnt, recv, roff, rcnt) -> list:
        self.C.xcomm_exchange(self.handle, int(slot), send, soff, scnt, recv, roff, rcnt)
        return [_NativeWork(self, int(slot))]

    def healthy(self) -> bool:
        return self.C.xcomm_async_error(self.handle) == 0

    def close(self) -> None:
        if self.handle:
            self.C.xcomm_destroy(self.handle)
            self.handle = 0


_NATIVE = {}


def native_exchange(ctx: Context) -> NativeExchange | None:
    """The job's NativeExchange (created on first call), or None when the backend is not RCCL, the context is a test
    transport (LazyContext) or PCMX_NATIVE_EXCHANGE=0."""
    if ctx.backend != "nccl" or isinstance(ctx, LazyContext) or os.environ.get("PCMX_NATIVE_EXCHANGE", "1") == "0":
        return None
    key = ctx.device.index
    if key not in _NATIVE:
        try:
            _NATIVE[key] = NativeExchange(ctx)
        except RuntimeError as e:  # (the same outcome on every rank: the probe's result is agreed)
            import sys

            print(f"[dist] {e}: exchanges go through torch.distributed", file=sys.stderr, flush=True)
            _NATIVE[key] = None
    return _NATIVE[key]


def native_exchange_active(ctx: Context) -> bool:
    """True when this job's exchanges run on the native RCCL communicator (reported in the bench line)."""
    return _NATIVE.get(ctx.device.index) is not None


class _DeferredWork:
    """An exchange whose data lands in its receive tensors only when waited on."""

    def __init__(self, pairs):
        self.pairs = pairs

    def wait(self):
        for dst, src in self.pairs:
            dst.copy_(src)
        self.pairs = []


class LazyContext(Context):
    """Test transport: exchange() moves the data at once into private buffers (the send tensors are copied when the
    exchange is posted, as a real transport reads them) but writes the receive tensors only in wait(). The worst case
    a real async transport allows — nothing arrives before it is waited for — every time: a schedule that reads an
    exchange's destination before waiting for it reads stale data deterministically (tests of the deferred SpMV
    pipeline, tests/test_parallel_cpu.py, tests/test_gpu_multi.py)."""

    def exchange(self, outs: list, ins: list, async_op: bool = False) -> list:
        tmp = [torch.empty_like(o) for o in outs]
        Context.exchange(self, tmp, [t.clone() for t in ins], async_op=False)
        w = _DeferredWork(list(zip(outs, tmp)))
        if async_op:
            return [w]
        w.wait()
        return []

    @staticmethod
    def of(ctx: Context) -> LazyContext:
        return LazyContext(ctx.rank, ctx.world, ctx.local_rank, ctx.device, ctx.backend)


_OPS = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}


def init(backend: str | None = None, device: str | None = None) -> Context:
    """Initialise from torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).

    backend: "nccl" (RCCL, default when a GPU is visible) or "gloo" (CPU tensors, or CUDA tensors with host-staged
    messages: several ranks can then share ONE GPU, which tests the N > 1 GPU paths on a 1-GPU box)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available() if device is None else device.startswith("cuda")
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": dev} if backend == "nccl" else {}
        # a collective that one rank never joins (it failed before reaching it) ends the job after this many
        # seconds (RCCL watchdog / gloo timeout) instead of hanging it
        kw["timeout"] = timedelta(seconds=int(os.environ.get("PCMX_PG_TIMEOUT_S", "600")))
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return Context(rank, world, local, dev, backend if world > 1 else "none")


def side_group(ctx: Context):
    """A CPU (gloo) process group beside the data group, for collective DECISIONS (did any rank fail a section?):
    its operations have their own sequence, so a decision can never pair with a data collective another rank is
    still waiting in. None when not distributed."""
    if not ctx.distributed:
        return None
    return dist.new_group(backend="gloo")


def gather_objects(obj, group=None) -> list:
    """Every rank's `obj` (picklable), in rank order, over `group` (a side_group; [obj] when not distributed)."""
    if group is None:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj, group=group)
    return out


def finalize(ctx: Context | None = None) -> None:
    if dist.is_initialized():
        try:
            if ctx is not None:
                ctx.barrier()
            if ctx is not None and ctx.device.type == "cuda":
                torch.cuda.synchronize(ctx.device)
            for nx in _NATIVE.values():
                if nx is not None:
                    nx.close()
            _NATIVE.clear()
        finally:
            dist.destroy_process_group()


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn_entry(rank, fn, world, port, backend, args):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    ctx = init(backend=backend, device="cpu" if backend == "gloo" else None)
    try:
        fn(ctx, *args)
    finally:
        finalize(ctx)


def spawn(fn, world: int, backend: str = "gloo", args: tuple = ()) -> None:
    """Run fn(ctx, *args) in `world` local processes (CPU/gloo test harness; rendezvous on 127.0.0.1)."""
    import torch.multiprocessing as mp

    mp.spawn(_spawn_entry, args=(fn, world, free_port(), backend, args), nprocs=world, join=True)
