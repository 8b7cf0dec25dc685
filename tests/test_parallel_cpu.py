"""Distributed layer on the CPU (gloo backend, real multi-process rendezvous on 127.0.0.1).

The same code paths run over RCCL on MI355X; here every distributed result is compared with the
single-process oracle of the same operation (SURVEY §4 strategy: golden outputs + independent models).
"""
import numpy as np
import pytest
import torch
from conftest import ASSETS, run_cli

from parallel_c_programs_amd import ops
from parallel_c_programs_amd.parallel import (CartTopology, DistributedSpMV, HaloExchanger2D, LazyContext, StencilSlab,
                                              dims_create, global_reduce, global_scan, grow_distributed,
                                              nnz_balanced_cuts, reference_run, spawn, split, token_ring)
from parallel_c_programs_amd.utils import bmp


# ------------------------------------------------------------------ pure topology (no processes)

@pytest.mark.parametrize("n,dims", [(1, [1, 1]), (2, [2, 1]), (4, [2, 2]), (6, [3, 2]), (8, [4, 2]), (12, [4, 3]),
                                    (16, [4, 4]), (7, [7, 1])])
def test_dims_create_matches_mpi(n, dims):
    assert dims_create(n) == dims


def test_cart_topology_tiles_cover_image():
    for world in (1, 2, 3, 4, 8):
        topo = CartTopology.create(world)
        H, W = 37, 53
        cover = np.zeros((H, W), dtype=int)
        for r in range(world):
            r0, r1, c0, c1 = topo.tile(r, H, W)
            cover[r0:r1, c0:c1] += 1
            nb = topo.neighbours(r)
            row, col = topo.coords(r)
            assert nb["north"] == (topo.rank_of(row - 1, col))
            if nb["east"] >= 0:
                assert topo.coords(nb["east"]) == (row, col + 1)
        assert (cover == 1).all()


def test_split_balanced():
    sizes = [split(10, 4, i) for i in range(4)]
    assert sizes == [(0, 3), (3, 6), (6, 8), (8, 10)]


def test_nnz_cuts_balance():
    rp = ops.sparse.powerlaw_row_ptr(20000, 400000)
    cuts = nnz_balanced_cuts(rp, 4)
    nnz = [int(rp[cuts[i + 1]] - rp[cuts[i]]) for i in range(4)]
    assert cuts[0] == 0 and cuts[-1] == 20000
    assert max(nnz) < 1.25 * (sum(nnz) / 4)


def test_powerlaw_rows_bit_identical():
    full = ops.powerlaw_csr(5000, 60000, seed=3)
    part = ops.sparse.powerlaw_csr_rows(full.row_ptr, 1200, 3100, 5000, seed=3)
    a, b = int(full.row_ptr[1200]), int(full.row_ptr[3100])
    assert torch.equal(part.col, full.col[a:b]) and torch.equal(part.val, full.val[a:b])


# ------------------------------------------------------------------ multi-process (gloo)

def _ring(ctx, out_q):
    out_q.put((ctx.rank, token_ring(ctx, verbose=False)))


class _Out:
    """Per-rank result sink backed by files (a pipe-backed queue would block writers of large results
    until the parent reads, but the parent only reads after the ranks are joined)."""

    def __init__(self, d):
        self.d = d

    def put(self, kv):
        import pickle

        k, v = kv
        with open(f"{self.d}/{k}.pkl", "wb") as f:
            pickle.dump(v, f)


def _collect(world, fn, *args):
    import os
    import pickle
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        spawn(fn, world, "gloo", (_Out(d), *args))
        res = {}
        for name in os.listdir(d):
            with open(os.path.join(d, name), "rb") as f:  # files written by this test's own ranks
                res[int(name.split(".")[0])] = pickle.load(f)
    return res


def test_token_ring_world4():
    res = _collect(4, _ring)
    assert res[0] == 2 * 4 - 2
    assert res[3] == 3  # top of the chain: received 3, no increment after


def _halo(ctx, q):
    topo = CartTopology.create(ctx.world)
    H, W = 12, 10
    full = torch.arange(H * W, dtype=torch.float32).view(H, W)
    r0, r1, c0, c1 = topo.tile(ctx.rank, H, W)
    padded = torch.nn.functional.pad(full, (1, 1, 1, 1), value=-1.0)
    tile = torch.full((r1 - r0 + 2, c1 - c0 + 2), -1.0)
    tile[1:-1, 1:-1] = full[r0:r1, c0:c1]
    HaloExchanger2D(ctx, topo).exchange_(tile)
    expect = padded[r0:r1 + 2, c0:c1 + 2].clone()
    # corners are not exchanged (4-connectivity); compare edges only
    for t in (tile, expect):
        t[0, 0] = t[0, -1] = t[-1, 0] = t[-1, -1] = 0
    q.put((ctx.rank, bool(torch.equal(tile, expect))))


@pytest.mark.parametrize("world", [2, 4])
def test_halo_exchange_matches_padded_slices(world):
    res = _collect(world, _halo)
    assert all(res.values()) and len(res) == world


def _exchange(ctx, q):
    """Context.exchange: a dense all-to-all with uneven and zero-size entries (self included), then a
    neighbour_exchange in which rank 0 has NO pairs (it must still enter the collective), then a duplicate peer."""
    W, r = ctx.world, ctx.rank
    ins = [torch.full((q_ * 2 + r,), float(100 * r + q_)) for q_ in range(W)]  # entry for q: 2q + r values
    outs = [torch.empty(2 * r + q_) for q_ in range(W)]                       # from q: 2r + q values
    ctx.exchange(outs, ins)
    ok = all(torch.equal(outs[q_], torch.full((2 * r + q_,), float(100 * q_ + r))) for q_ in range(W))
    # ring neighbour exchange among ranks 1..W-1 only; rank 0 passes an empty list
    pairs = []
    if r > 0:
        nxt, prv = 1 + (r % (W - 1)), 1 + ((r - 2) % (W - 1))
        pairs = [(nxt, torch.tensor([float(r)]), torch.empty(1))]
        if prv != nxt:
            pairs.append((prv, torch.tensor([float(r)]), torch.empty(1)))
    ctx.neighbour_exchange(pairs)
    ok &= all(float(rcv) == float(p) for p, _, rcv in pairs)
    try:
        ctx.neighbour_exchange([(0, torch.zeros(1), torch.zeros(1))] * 2)
        ok = False
    except ValueError:
        pass
    q.put((r, bool(ok)))


@pytest.mark.parametrize("world", [3, 4])
def test_context_exchange_uneven_empty_and_no_pairs(world):
    res = _collect(world, _exchange)
    assert len(res) == world and all(res.values()), res


def _reduce_scan(ctx, q):
    g = torch.Generator().manual_seed(10 + ctx.rank)
    x = torch.rand(1000 + 37 * ctx.rank, generator=g)
    s = global_reduce(x, ctx)
    mx = global_reduce(x, ctx, "max")
    y = global_scan(x, ctx)
    q.put((ctx.rank, (float(s), float(mx), y.numpy(), x.numpy())))


def test_global_reduce_and_scan_world3():
    res = _collect(3, _reduce_scan)
    xs = [torch.from_numpy(res[r][3]) for r in range(3)]
    cat = torch.cat(xs).double()
    for r in range(3):
        assert abs(res[r][0] - cat.sum().item()) < 1e-3
        assert res[r][1] == pytest.approx(cat.max().item())
    ys = torch.cat([torch.from_numpy(res[r][2]) for r in range(3)]).double()
    assert torch.allclose(ys, torch.cumsum(cat, 0), rtol=1e-5, atol=1e-3)


def _reduce_overlap(ctx, q):
    """Reduce workload: each step's all-reduce stays in flight behind the next step (round 6)."""
    from parallel_c_programs_amd.models import workloads as W

    w = W.Reduce(ctx, n=5000)
    inflight = []
    for _ in range(3):
        w.step()
        inflight.append(w._pending is not None)
    c = w.check(reduce=True)
    q.put((ctx.rank, (inflight, w._pending is None, float(w.total), c["check_passed"], float(w.x.double().sum()))))


def test_reduce_workload_overlapped_allreduce_world2():
    res = _collect(2, _reduce_overlap)
    total = sum(res[r][4] for r in range(2))
    for r in range(2):
        inflight, settled, got, passed, _ = res[r]
        assert inflight == [True, True, True] and settled and passed
        assert abs(got - total) <= 1e-5 * total


def _scan_turns(ctx, q):
    from parallel_c_programs_amd.models import workloads as W

    w = W.Scan(ctx, n=3000)
    w.step()
    a = w.check(reduce=True, chunk=1000)
    b = w.check(reduce=True, chunk=1000, one_rank_at_a_time=True)
    q.put((ctx.rank, (a["check_passed"], b["check_passed"], a["rel_err_vs_fp64"], b["rel_err_vs_fp64"])))


def test_scan_check_one_rank_at_a_time_world3():
    """The shared-GPU form of the scan check (ranks take turns for the fp64 cumsums) gives the same verdict."""
    res = _collect(3, _scan_turns)
    for r in range(3):
        pa, pb, ea, eb = res[r]
        assert pa and pb and ea == eb


def _region(ctx, q, path):
    img = torch.from_numpy(bmp.read(path)) if ctx.is_root else None
    stats = {}
    reg = grow_distributed(ctx, img, 2, stats=stats)
    if ctx.is_root:
        q.put((0, (reg.numpy(), stats)))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_distributed_region_equals_serial(world):
    path = str(ASSETS / "pic1.bmp")
    res = _collect(world, _region, path)
    reg, stats = res[0]
    reg = torch.from_numpy(reg)
    img = torch.from_numpy(bmp.read(path))
    serial = ops.region2d(img)
    assert torch.equal(reg, serial)
    assert stats["outer_steps"] >= 2  # the region crosses tile borders


def _stencil(ctx, q, n, cols, steps, overlap, fuse=1, halo_mult=1):
    slab = StencilSlab(ctx, n, cols, fuse=fuse, halo_mult=halo_mult)
    slab.run(steps, overlap)
    full = slab.gather()
    if ctx.is_root:
        q.put((0, full.view(torch.int16).numpy()))


@pytest.mark.parametrize("world,overlap", [(2, True), (3, False), (4, True)])
def test_distributed_stencil_bit_exact(world, overlap):
    n, cols, steps = 64, 48, 7
    res = _collect(world, _stencil, n, cols, steps, overlap)
    ref = reference_run(n, steps, cols)
    assert torch.equal(torch.from_numpy(res[0]), ref.view(torch.int16))


@pytest.mark.parametrize("world,overlap,fuse", [(1, True, 2), (2, True, 2), (3, False, 2), (4, True, 2), (2, True, 4),
                                                (3, True, 3)])
def test_distributed_stencil_fused_steps_bit_exact(world, overlap, fuse):
    """Temporal blocking: `fuse`-row halos, one exchange per `fuse` updates, same bits as single steps."""
    n, cols, steps = 64, 48, 12
    res = _collect(world, _stencil, n, cols, steps, overlap, fuse)
    ref = reference_run(n, steps, cols)
    assert torch.equal(torch.from_numpy(res[0]), ref.view(torch.int16))


@pytest.mark.parametrize("world,overlap,fuse,m,steps", [(2, True, 2, 2, 12), (3, True, 2, 3, 10), (4, True, 4, 2, 16),
                                                        (3, False, 3, 2, 9), (2, True, 4, 3, 12)])
def test_distributed_stencil_deep_halo_bit_exact(world, overlap, fuse, m, steps):
    """Deep halo: m*fuse halo rows exchanged every m steps, the rows next to a neighbour recomputed in between (one
    exchange + one edge launch per m steps) — same bits as single steps, also when the run stops mid-period."""
    n, cols = 72, 40
    res = _collect(world, _stencil, n, cols, steps, overlap, fuse, m)
    ref = reference_run(n, steps, cols)
    assert torch.equal(torch.from_numpy(res[0]), ref.view(torch.int16))


def _stencil_ckpt(ctx, q, prefix):
    a = StencilSlab(ctx, 40, 24)
    a.run(4)
    a.checkpoint(prefix)
    a.run(3)
    b = StencilSlab(ctx, 40, 24)
    b.restore(prefix)
    b.run(3)
    fa, fb = a.gather(), b.gather()
    if ctx.is_root:
        q.put((0, (fa.view(torch.int16).numpy(), fb.view(torch.int16).numpy(), b.steps_done)))


def test_stencil_checkpoint_resume_world2(tmp_path):
    res = _collect(2, _stencil_ckpt, str(tmp_path / "ck"))
    fa, fb, steps = res[0]
    assert steps == 7 and np.array_equal(fa, fb)
    assert np.array_equal(fa, reference_run(40, 7, 24).view(torch.int16).numpy())


def _spmv(ctx, q, n, nnz, chunks, exchange, colsplit=None, chunk0_frac=None):
    d = DistributedSpMV.powerlaw(ctx, n, nnz, seed=1, chunks=chunks, exchange=exchange, colsplit=colsplit,
                                 chunk0_frac=chunk0_frac)
    x = torch.linspace(0, 1, n)
    y = d.step(x)
    y2 = d.step(y / y.abs().max())
    # fast path: iterate in the rank's layout (ghost segments / padded all-gather slots filled in place)
    xp = d.to_padded(x)
    yp = d.step_padded(xp)
    yp2 = d.step_padded(yp / yp.abs().max())
    ids = d.layout_ids()
    q.put((ctx.rank, (y.numpy(), y2.numpy(), d.from_padded(yp2).numpy(), d.n_pad, ids.numpy(), yp2.numpy(),
                      d.colsplit)))


@pytest.mark.parametrize("exchange", ["ghost", "allgather"])
@pytest.mark.parametrize("world,chunks", [(3, 1), (3, 4), (2, 3), (4, 2)])
def test_distributed_spmv_matches_serial(world, chunks, exchange):
    n, nnz = 3000, 40000
    res = _collect(world, _spmv, n, nnz, chunks, exchange)
    m = ops.powerlaw_csr(n, nnz, seed=1)
    x = torch.linspace(0, 1, n)
    y = ops.spmv(m, x)
    y2 = ops.spmv(m, y / y.abs().max())
    for r in range(world):
        assert not res[r][6]  # the column split is a GPU (sliced) default only
        assert torch.equal(torch.from_numpy(res[r][0]), y)  # same rows, same kernel: bit-identical
        assert torch.allclose(torch.from_numpy(res[r][1]), y2, rtol=1e-5, atol=1e-5)
        assert torch.allclose(torch.from_numpy(res[r][2]), y2, rtol=1e-5, atol=1e-5)
        # every layout entry (own rows and the ghosts / replicas the exchange delivered) holds y2 of its row
        ids, yp2 = torch.from_numpy(res[r][4]), torch.from_numpy(res[r][5])
        assert torch.allclose(yp2[ids >= 0], y2[ids[ids >= 0]], rtol=1e-5, atol=1e-5)
        if exchange == "allgather":
            assert res[r][3] >= n
        else:  # compact: own rows + the ghosts its nonzeros reference, never more than the whole vector
            assert res[r][3] <= n and int((ids >= 0).sum()) == res[r][3]


@pytest.mark.parametrize("world", [2, 4])
def test_distributed_spmv_colsplit_plain_csr(world):
    """The column-split schedule on the plain CSR path (ColSplitCSR, asked for explicitly): (A_<B x) + (A_>=B x) is
    another fp32 summation order, so it matches the serial product to rounding, not bit for bit."""
    n, nnz = 3000, 40000
    res = _collect(world, _spmv, n, nnz, 2, "ghost", True)
    m = ops.powerlaw_csr(n, nnz, seed=1)
    x = torch.linspace(0, 1, n)
    y = ops.spmv(m, x)
    y2 = ops.spmv(m, y / y.abs().max())
    for r in range(world):
        assert res[r][6]
        assert torch.allclose(torch.from_numpy(res[r][0]), y, rtol=1e-5, atol=1e-5)
        ids, yp2 = torch.from_numpy(res[r][4]), torch.from_numpy(res[r][5])
        assert torch.allclose(yp2[ids >= 0], y2[ids[ids >= 0]], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("world,colsplit,frac", [(2, False, 0.3), (4, True, 0.35), (4, False, 0.7)])
def test_distributed_spmv_uneven_row_chunks(world, colsplit, frac):
    """Uneven row chunks (round 6: chunk 0 takes `frac` of each rank's rows, so the column-split step posts chunk 0's
    smaller exchange earlier): the same rows through the same kernel give the serial product bit for bit, and every
    layout entry (own rows and the ghosts the uneven exchanges delivered) holds its row's value."""
    n, nnz = 3000, 40000
    res = _collect(world, _spmv, n, nnz, 2, "ghost", colsplit, frac)
    m = ops.powerlaw_csr(n, nnz, seed=1)
    x = torch.linspace(0, 1, n)
    y = ops.spmv(m, x)
    y2 = ops.spmv(m, y / y.abs().max())
    for r in range(world):
        assert res[r][6] == colsplit
        if colsplit:
            assert torch.allclose(torch.from_numpy(res[r][0]), y, rtol=1e-5, atol=1e-5)
        else:
            assert torch.equal(torch.from_numpy(res[r][0]), y)
        ids, yp2 = torch.from_numpy(res[r][4]), torch.from_numpy(res[r][5])
        assert torch.allclose(yp2[ids >= 0], y2[ids[ids >= 0]], rtol=1e-5, atol=1e-5)


def _spmv_chunk_bounds(ctx, q, frac):
    d = DistributedSpMV.powerlaw(ctx, 3000, 40000, seed=1, chunks=2, chunk0_frac=frac)
    q.put((ctx.rank, (d.cb, [d.chunk_rows(c) for c in range(2)], d.rows, d.block)))


def test_spmv_chunk0_frac_bounds_are_global():
    """The chunk boundaries are the same on every rank (fractions of the LARGEST block), so a ghost's chunk is known
    to its receiver without asking its owner."""
    res = _collect(3, _spmv_chunk_bounds, 0.3)
    cbs = {tuple(res[r][0]) for r in range(3)}
    assert len(cbs) == 1
    cb = cbs.pop()
    block = res[0][3]
    assert cb[0] == 0 and cb[1] == round(0.3 * block) and cb[2] >= block
    for r in range(3):
        (a0, b0), (a1, b1) = res[r][1]
        assert a0 == 0 and b0 == a1 and b1 == res[r][2]


def _late_wait_colsplit(self, xp, out):
    """_step_colsplit with the previous step's chunk-1 wait moved AFTER the chunk-1-column products (a bug)."""
    W, r = self.ctx.world, self.ctx.rank
    self._wait(0)
    for c, (a, b, part) in enumerate(self.parts):
        if b > a:
            part.product_phase(xp, 0, c)
    pending = [[], []]
    for c, (a, b, part) in enumerate(self.parts):
        s0 = self.seg[c * W + r]
        if b > a:
            part.product_phase(xp, 1, c, out[s0:s0 + (b - a)])
        pending[c] = self._post_chunk(out, c)
    self._wait(1)
    self._pending = pending
    return out


def _spmv_iterate(ctx, q, n, nnz, steps, buggy):
    d = DistributedSpMV.powerlaw(LazyContext.of(ctx), n, nnz, seed=1, chunks=2, colsplit=True)
    if buggy:
        d._step_colsplit = _late_wait_colsplit.__get__(d)
    xp = d.to_padded(torch.linspace(0, 1, n))
    err = d.iterate_max_rel_err(xp, steps, defer=True)
    y = d.from_padded(d.iterate(xp, steps, defer=True))
    q.put((ctx.rank, (err, y.numpy(), d.colsplit)))


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("buggy", [False, True])
def test_distributed_spmv_deferred_pipeline_iterates(world, buggy):
    """The steady-state pipeline as an ITERATION: K = 5 chained steps x <- A x with each step's chunk-1 exchange left
    in flight into the next step (deferred), through a transport that delivers only on wait, against the serial fp64
    A^K x. A schedule that waits for the chunk-1 exchange after the products that read it must fail."""
    n, nnz, K = 3000, 40000, 5
    res = _collect(world, _spmv_iterate, n, nnz, K, buggy)
    m = ops.powerlaw_csr(n, nnz, seed=1)
    A = torch.sparse_csr_tensor(m.row_ptr, m.col.long(), m.val.double(), size=(n, n))
    ref = torch.linspace(0, 1, n).double()
    for _ in range(K):
        ref = A @ ref
    for r in range(world):
        err, y, split = res[r]
        assert split
        full_err = (torch.from_numpy(y).double() - ref).abs().max().item() / ref.abs().max().item()
        if buggy:
            assert err > 1e-3 and full_err > 1e-3, (err, full_err)
        else:
            assert err < 1e-5 and full_err < 1e-5, (err, full_err)


def _spmv_uneven(ctx, q, cuts, chunks, exchange):
    from parallel_c_programs_amd.ops.sparse import powerlaw_csr_rows, powerlaw_row_ptr

    n = cuts[-1]
    rp = powerlaw_row_ptr(n, 30000, 2.5, 3)
    local = powerlaw_csr_rows(rp, cuts[ctx.rank], cuts[ctx.rank + 1], n, 3)
    d = DistributedSpMV(ctx, rp, local, cuts, chunks=chunks, exchange=exchange)
    x = torch.linspace(0, 1, n)
    y = d.step(x)
    xp = d.to_padded(x)
    y2 = d.from_padded(d.step_padded(d.step_padded(xp)))
    q.put((ctx.rank, (y.numpy(), y2.numpy(), d.colsplit)))


@pytest.mark.parametrize("exchange", ["ghost", "allgather"])
@pytest.mark.parametrize("cuts,chunks", [([0, 0, 1200, 2000], 2), ([0, 700, 700, 2000], 3), ([0, 5, 1990, 2000], 4)])
def test_distributed_spmv_uneven_and_empty_ranks(cuts, chunks, exchange):
    """Row blocks of very different sizes, an EMPTY rank (no rows: no products, empty sends, still part of every
    collective) and more chunks than a small rank has rows: the exchange still delivers every referenced entry."""
    res = _collect(len(cuts) - 1, _spmv_uneven, cuts, chunks, exchange)
    from parallel_c_programs_amd.ops.sparse import powerlaw_csr_rows, powerlaw_row_ptr

    n = cuts[-1]
    m = powerlaw_csr_rows(powerlaw_row_ptr(n, 30000, 2.5, 3), 0, n, n, 3)
    x = torch.linspace(0, 1, n)
    y = ops.spmv(m, x)
    y2 = ops.spmv(m, ops.spmv(m, x))
    for r in range(len(cuts) - 1):
        assert not res[r][2]
        assert torch.equal(torch.from_numpy(res[r][0]), y)
        assert torch.allclose(torch.from_numpy(res[r][1]), y2, rtol=1e-5, atol=1e-4)


def test_padded_index_is_a_permutation_and_identity_on_one_rank():
    from parallel_c_programs_amd.parallel.spmv import padded_index

    assert torch.equal(padded_index([0, 1000], 1, 1000), torch.arange(1000))
    assert torch.equal(padded_index([0, 1000], 3, 334), torch.arange(1000))
    cuts, C = [0, 7, 7, 20, 31], 3  # an empty rank, uneven blocks
    L = -(-13 // C)
    p = padded_index(cuts, C, L)
    assert p.unique().numel() == 31 and int(p.max()) < C * 4 * L
    # chunk c of rank r is the contiguous all-gather slot [c*W*L + r*L, c*W*L + (r+1)*L)
    g = 7 + 5  # rank 2, local row 5 -> chunk 1 (L = 5), offset 0
    assert int(p[g]) == 1 * 4 * L + 2 * L + 0


def test_bench_rehearsal_gloo_world2():
    """The driver's N>1 bench path (every section, its checks and the JSON contract) under torchrun + gloo."""
    import json
    import subprocess
    import sys

    from conftest import ROOT, cli_env
    from parallel_c_programs_amd.parallel import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--small", "--device", "cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=cli_env(OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["value"] > 0
    for k in ("reduce_weak_gbps", "reduce_strong_gbps", "scan_weak_gbps", "scan_strong_gbps", "stencil_glups",
              "spmv_gflops"):
        assert out[k] > 0, k
    assert out["stencil_bit_exact"] and out["stencil_finite"]
    assert out["sgemm_max_rel_err_vs_fp64"] < 1e-5 and out["spmv_max_rel_err_vs_fp64"] < 1e-5
    assert out["reduce_strong_rel_err_vs_fp64"] < 1e-5 and out["scan_strong_rel_err_vs_fp64"] < 1e-5
    assert not [k for k in out if k.endswith("_error")]


def test_bench_failed_section_is_reported_and_fails_the_run():
    """A section that raises (here: an unsupported stencil fuse depth) costs only its own fields: the line still
    prints once, with "<section>_error", the later sections still run, and the run exits 1."""
    import json
    import subprocess
    import sys

    from conftest import ROOT, cli_env

    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--small", "--device", "cpu", "--steps", "1",
                        "--warmup", "0", "--sections", "stencil,spmv", "--stencil-fuse", "99"],
                       capture_output=True, text=True, timeout=300, env=cli_env(OMP_NUM_THREADS="2"))
    assert r.returncode == 1, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["stencil_error"].startswith("ValueError") and "stencil_glups" not in out
    assert out["spmv_gflops"] > 0 and out["spmv_max_rel_err_vs_fp64"] < 1e-5
    assert out["checks_passed"] is False


def _bench_cpu(*extra, timeout=600):
    """bench.py on the CPU WITHOUT a launcher (--gpus N > 1 makes it start torch.distributed.run itself)."""
    import json
    import subprocess
    import sys

    from conftest import ROOT, cli_env

    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--small", "--device", "cpu", *extra],
                       capture_output=True, text=True, timeout=timeout, env=cli_env(OMP_NUM_THREADS="1"))
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[0]) if len(lines) == 1 else None), len(lines)


def test_bench_gpus_2_launches_two_ranks_itself():
    """`bench.py --gpus 2` with no WORLD_SIZE: one torch.distributed.run child with 2 ranks, ONE line, n_gpus 2."""
    r, out, nlines = _bench_cpu("--gpus", "2", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-3000:]
    assert nlines == 1 and out["n_gpus"] == 2 and out["checks_passed"] is True
    assert out["config"]["parallelism"] == "dp2" and out["reduce_strong_gbps"] > 0
    for k in ("sgemm", "reduce_weak", "scan_weak", "stencil", "spmv"):
        assert out[f"{k}_device_ms_median"] > 0, k


@pytest.mark.parametrize("world", [2, 4])
def test_bench_n_gt_1_line_explains_itself(world):
    """At N > 1 every distributed section also times its compute-only twin in the same job: the
    line carries compute-only and exposed-communication ms, the per-rank spread of the median step time, the bytes
    exchanged per step (per rank and in total) and the process group's size, with every check passing."""
    r, out, nlines = _bench_cpu("--gpus", str(world), "--steps", "2", "--warmup", "1", "--no-x6")
    assert r.returncode == 0, r.stderr[-3000:]
    assert nlines == 1 and out["checks_passed"] is True
    assert out["comm_world_size"] == world and out["comm_backend"] == "gloo"
    for sec in ("reduce_weak", "reduce_strong", "scan_weak", "scan_strong", "stencil", "spmv"):
        assert out[f"{sec}_compute_only_ms"] > 0, sec
        full = out[f"{sec}_ms_per_step"]
        assert out[f"{sec}_comm_exposed_ms"] == pytest.approx(full - out[f"{sec}_compute_only_ms"], abs=2e-3), sec
        assert 0 < out[f"{sec}_rank_step_ms_min"] <= out[f"{sec}_rank_step_ms_max"], sec
        assert 0 < out[f"{sec}_compute_only_rank_ms_min"] <= out[f"{sec}_compute_only_rank_ms_max"], sec
        per, tot = out[f"{sec}_bytes_exchanged_per_step"], out[f"{sec}_bytes_exchanged_per_step_total"]
        assert 0 < per <= tot <= world * per, sec
    assert out["reduce_weak_bytes_exchanged_per_step_total"] == 4.0 * world
    # stencil: the interior ranks send `halo` bf16 rows of 256 columns to each of two neighbours every m steps
    m, T = out["stencil_halo_mult"], out["stencil_updates_per_step"]
    assert out["stencil_bytes_exchanged_per_step"] == (2 if world > 2 else 1) * m * T * 256 * 2 / m


@pytest.mark.parametrize("section,key", [("stencil", "stencil_halo_selftest_bit_exact"),
                                         ("spmv", "spmv_pipeline_selftest_bit_identical")])
def test_bench_failed_selftest_fails_the_section(section, key):
    """An N > 1 self-test that fails (deep halo / deferred SpMV pipeline) is a failed check of its section, not only
    a field of the line: the run exits 1 with the key in "<section>_check_failed"."""
    r, out, nlines = _bench_cpu("--gpus", "2", "--steps", "1", "--warmup", "0", "--sections", section,
                                "--inject-fault", f"{section}:1:selftest")
    assert r.returncode == 1, r.stderr[-3000:]
    assert nlines == 1 and out["checks_passed"] is False and out[key] is False
    assert out[f"{section}_check_failed"] == [key]


def test_bench_world_size_mismatch_is_an_error():
    import subprocess
    import sys

    from conftest import ROOT, cli_env
    from parallel_c_programs_amd.parallel import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "bench.py"), "--gpus", "3", "--small",
           "--device", "cpu", "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=cli_env(OMP_NUM_THREADS="1"))
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("fault,section,failed_key", [
    ("sgemm:1:perturb", "sgemm", "sgemm_max_rel_err_vs_fp64"),
    ("scan:0:perturb", "scan", "scan_weak_rel_err_vs_fp64"),
    ("axpy:1:perturb", "axpy", "axpy_rel_err_vs_fp64"),
    ("stencil:1:perturb", "stencil", "stencil_timed_grid_bit_exact"),
    ("spmv:1:perturb", "spmv", "spmv_max_rel_err_vs_fp64"),
])
def test_bench_wrong_result_on_one_rank_fails_the_run(fault, section, failed_key):
    """A wrong timed result on ONE rank (injected after timing): every rank records the failed check in the same
    collective decision, the line still prints once with "<section>_check_failed", the later sections still run,
    and the run exits 1 (ref 3-serial-optimization/spmv.c:179-191, 366: every output compared)."""
    r, out, nlines = _bench_cpu("--gpus", "2", "--steps", "1", "--warmup", "0", "--inject-fault", fault)
    assert r.returncode == 1, r.stderr[-3000:]
    assert nlines == 1 and out["checks_passed"] is False
    assert failed_key in out[f"{section}_check_failed"]
    assert not [k for k in out if k.endswith("_check_failed") and k != f"{section}_check_failed"]
    assert out["spmv_gflops"] > 0 and out["value"] > 0


def test_bench_exception_on_one_rank_is_a_collective_decision():
    """A section that raises on rank 1 only (after its collectives): both ranks record "<section>_error", the
    following sections run on both ranks (no mismatched collectives, no hang) and pass, the run exits 1."""
    r, out, nlines = _bench_cpu("--gpus", "2", "--steps", "1", "--warmup", "0", "--inject-fault", "reduce:1:raise")
    assert r.returncode == 1, r.stderr[-3000:]
    assert nlines == 1 and out["reduce_error"].startswith("rank 1: RuntimeError")
    assert out["scan_strong_rel_err_vs_fp64"] < 1e-5 and out["stencil_bit_exact"] and out["spmv_gflops"] > 0
    assert not [k for k in out if k.endswith("_check_failed")]


@pytest.mark.parametrize("section", ["stencil", "spmv"])
def test_bench_early_exception_on_one_rank_does_not_hang(section):
    """A section that raises on rank 1 right after its set-up, BEFORE its timed region (whose barriers rank 0 would
    otherwise wait in until the process-group timeout): rank 0 stops at the next decision point, both ranks record
    "<section>_error" from rank 1, the later sections run, the run exits 1 — well inside the test's time limit."""
    r, out, nlines = _bench_cpu("--gpus", "2", "--steps", "1", "--warmup", "0", "--inject-fault",
                                f"{section}:1:raise-early", timeout=300)
    assert r.returncode == 1, r.stderr[-3000:]
    assert nlines == 1 and out[f"{section}_error"].startswith("rank 1: RuntimeError: injected"), out
    assert out["checks_passed"] is False and out["value"] > 0
    assert f"{section}_glups" not in out and f"{section}_gflops" not in out
    if section == "stencil":
        assert out["spmv_gflops"] > 0 and out["spmv_max_rel_err_vs_fp64"] < 1e-5


def test_bench_under_launcher_without_gpus_flag():
    """torchrun --nproc-per-node 2 bench.py (no --gpus): the launcher's WORLD_SIZE is the rank count."""
    import json
    import subprocess
    import sys

    from conftest import ROOT, cli_env
    from parallel_c_programs_amd.parallel import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "bench.py"), "--small", "--device", "cpu",
           "--steps", "1", "--warmup", "0", "--sections", "reduce"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=cli_env(OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 2 and out["reduce_strong_gbps"] > 0


# ------------------------------------------------------------------ launcher-level (torch.distributed.run)

def _torchrun(nproc, module, *args):
    import subprocess
    import sys

    from conftest import cli_env
    from parallel_c_programs_amd.parallel import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m",
           f"parallel_c_programs_amd.cli.{module}", *map(str, args)]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=cli_env(OMP_NUM_THREADS="1"))


def test_cli_region_torchrun_writes_golden(tmp_path):
    r = _torchrun(4, "run_region", ASSETS / "pic1.bmp", "--backend", "gloo")
    assert r.returncode == 0, r.stderr[-2000:]
    out = bmp.read(tmp_path / "out.bmp")
    golden = bmp.read(ASSETS / "region_pic1_golden.bmp")
    assert np.array_equal(out, golden)


def test_cli_mpi_ring_prints_reference_lines():
    r = _torchrun(3, "run_mpi_ring", "--backend", "gloo")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = set(r.stdout.splitlines())
    for want in ["Rank 0 sent 0 ", "Rank 1 received 0 ", "Rank 1 sent 1 ", "Rank 2 received 1 ",
                 "Rank 2 sent 2 ", "Rank 1 received 2 ", "Rank 1 sent 3 ", "Rank 0 received 3 "]:
        assert want in lines


def test_cli_region_usage_message():
    r = run_cli("run_region", check=False)
    assert r.stdout == "Useage: region file" and r.returncode == 255


# ------------------------------------------------------------------ 3-D pipeline, z-slabs

def _volume3d(ctx, q):
    import hashlib

    from parallel_c_programs_amd.parallel import DistributedVolume

    dv = DistributedVolume(ctx, 512)
    n = torch.tensor([dv.grow()], dtype=torch.int64)
    ctx.all_reduce_(n)
    img = dv.raycast(64)
    reg = dv.gather_region()
    if ctx.is_root:
        digest = hashlib.md5(reg.numpy().tobytes()).hexdigest()
        q.put((0, (int(n), img.numpy(), int(reg.sum()), digest, dv.stats)))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_distributed_volume_zslabs_match_single_volume(world):
    """z-slab region growing (halo planes, device-style termination) and the pipelined slab ray caster reproduce
    the single-volume T2 region (2,197,899 voxels) and a bit-identical 64x64 reference image."""
    import hashlib

    vol = ops.create_volume(512, device="cpu", seed=0)
    reg_ref, _ = ops.region3d(vol)
    img_ref = ops.raycast(vol, reg_ref, 64, method="global")
    res = _collect(world, _volume3d)
    n, img, nreg, digest, stats = res[0]
    assert n == 2197899 and nreg == 2197899
    assert digest == hashlib.md5(reg_ref.numpy().tobytes()).hexdigest()
    assert np.array_equal(img, img_ref.numpy())
    assert stats["host_reads"] <= stats["outer_steps"] // 2 + 1


# ------------------------------------------------------------------ run_workload numerics checks (exit 1 on failure)

@pytest.mark.parametrize("name,sets", [
    ("region2d", []), ("region2d", ["side=700"]), ("histeq", ["side=512"]), ("region3d", []),
    ("raycast", ["image_dim=32", "method=global"]),
])
def test_run_workload_checks_pass_on_cpu(name, sets):
    """Every workload carries a real check: region2d = the golden out.bmp (T1) / the serial oracle, histeq = the
    serial host oracle bit for bit (T3), region3d = the 2,197,899-voxel box (T2), raycast = the serial caster."""
    import json

    args = [name, "--steps", "1", "--warmup", "0", "--device", "cpu"]
    for s_ in sets:
        args += ["--set", s_]
    r = run_cli("run_workload", *args, check=False, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["check_passed"] is True, out


def test_run_workload_failed_check_exits_1(monkeypatch):
    """A wrong result fails the check: the line is printed with check_passed false and the process exits 1."""
    from parallel_c_programs_amd.cli import run_workload
    from parallel_c_programs_amd.models import workloads as W

    real = W.Histeq.step

    def broken(self):
        real(self)
        self.out = self.out.clone()
        self.out.view(-1)[5] ^= 1

    monkeypatch.setattr(W.Histeq, "step", broken)
    with pytest.raises(SystemExit) as e:
        run_workload.run("histeq", ["--steps", "1", "--warmup", "0", "--device", "cpu", "--set", "side=64"])
    assert e.value.code == 1


def test_auto_halo_mult_rule():
    """Deep halo m = 5 on distributed slabs of up to 4096 rows (the N = 8 and N = 4 ranks of the 16384-row bench
    grid), else 1."""
    from parallel_c_programs_amd.parallel.stencil import auto_halo_mult

    assert auto_halo_mult(2048, 6, 8) == 5 and auto_halo_mult(2048, 8, 8) == 5
    assert auto_halo_mult(3072, 6, 4) == 5 and auto_halo_mult(4096, 6, 4) == 5
    assert auto_halo_mult(6144, 8, 3) == 1 and auto_halo_mult(8192, 8, 2) == 1  # taller slabs: m = 1
    assert auto_halo_mult(2048, 6, 1) == 1  # one rank: no exchange to amortise
    assert auto_halo_mult(2048, 1, 8) == 1  # single-step launches
    assert auto_halo_mult(50, 6, 8) == 1  # slab shorter than 10 fused levels (two 5T halos)


def test_gather_host_path_matches_index():
    """ops.gather_ (the SpMV send-buffer pack) on the host: out[i] = src[idx[i]] with int32 indices."""
    g = torch.Generator().manual_seed(3)
    src = torch.rand(1000, generator=g)
    idx = torch.randint(0, 1000, (257,), generator=g, dtype=torch.int32)
    out = torch.empty(257)
    ops.gather_(src, idx, out)
    assert torch.equal(out, src[idx.long()])


def _rocsparse_ranks(ctx, q, fail_rank):
    """bench.rocsparse_bar_ranks with the child process replaced: rank r 'measures' (r + 1) ms for csr_adaptive and
    2 (r + 1) ms for csr_rowsplit on (r + 1) * 1e6 nonzeros; `fail_rank`'s child fails."""
    import bench

    def fake(n_rows, nnz, reps, warmup, rows=None, device=None):
        r = ctx.rank
        if r == fail_rank:
            return {"rocsparse_spmv_gflops": "failed: RuntimeError: boom"}
        return {"rocsparse_spmv_gflops": 1.0, "rocsparse_spmv_max_rel_err_vs_fp64": 1e-7 * (r + 1),
                "_ms": {"csr_adaptive": float(r + 1), "csr_rowsplit": 2.0 * (r + 1)}, "_nnz": (r + 1) * 1_000_000}

    bench.rocsparse_bar = fake
    bench.torch.cuda.device_count = lambda: ctx.world if fail_rank != -2 else 1  # one GPU per rank (-2: shared)
    q.put((ctx.rank, bench.rocsparse_bar_ranks(ctx, 100, 100, 1, 0, (0, 1))))


def test_rocsparse_bar_ranks_takes_the_slowest_rank():
    """N > 1 vendor bar: per algorithm the slowest rank's time, over the whole matrix's nonzeros (sum over ranks), the
    best algorithm; every rank makes the same collectives, also when one rank's child process failed."""
    res = _collect(2, _rocsparse_ranks, -1)
    # nnz 3e6 over the slower rank's 2 ms (adaptive) / 4 ms (rowsplit): 3 / 1.5 GFLOP/s
    assert res[0] == res[1]
    assert res[0]["rocsparse_spmv_alg"] == "csr_adaptive" and abs(res[0]["rocsparse_spmv_gflops"] - 3.0) < 1e-9
    assert abs(res[0]["rocsparse_spmv_max_rel_err_vs_fp64"] - 2e-7) < 1e-15
    res = _collect(2, _rocsparse_ranks, 1)  # rank 1 failed: its time counts as infinite -> no bar
    assert res[0] == res[1] and isinstance(res[0]["rocsparse_spmv_gflops"], str)
    res = _collect(2, _rocsparse_ranks, -2)  # two ranks on one GPU: no child processes at all
    assert res[0] == res[1] == {"rocsparse_spmv_gflops": "not measured: ranks share a GPU"}


def _timed_host(ctx, q):
    from parallel_c_programs_amd.utils.harness import timed

    calls, ms, hms = [], [], []
    timed(ctx, lambda: calls.append(1), 5, 2, ms, hms, settle_ms=50.0)
    q.put((ctx.rank, (len(calls), len(ms), len(hms))))


def test_timed_collects_host_times_and_settles_only_on_gpu():
    """timed(): W + K calls on the CPU (the settle phase is for the GPU clock only), per-step times and host enqueue
    times for every timed step."""
    res = _collect(2, _timed_host)
    assert res[0] == res[1] == (7, 5, 5)
