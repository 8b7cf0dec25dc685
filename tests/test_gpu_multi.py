"""Multi-process GPU paths: the bench contract on the GPU at one rank, and every north-star workload under
torchrun over RCCL on all visible GPUs (skipped on a 1-GPU box; the driver's 8-GPU node runs it)."""
import json
import subprocess
import sys

import numpy as np
import pytest
import torch
from conftest import ASSETS, ROOT, cli_env

from parallel_c_programs_amd.utils import bmp

pytestmark = pytest.mark.gpu


def _bench(nproc, *extra, timeout=240, self_launch=False):
    from parallel_c_programs_amd.parallel import free_port

    if nproc == 1 or self_launch:  # (bench.py --gpus N > 1 starts torch.distributed.run itself)
        cmd = [sys.executable, str(ROOT / "bench.py")]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "bench.py")]
    cmd += ["--gpus", str(nproc), *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=cli_env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _check_line(out, n):
    assert out["n_gpus"] == n and out["device"] == "cuda" and out["value"] > 0
    assert out["checks_passed"] is True and not [k for k in out if k.endswith("_check_failed")], out
    for k in ("reduce_weak_gbps", "reduce_strong_gbps", "scan_weak_gbps", "scan_strong_gbps", "stencil_glups",
              "spmv_gflops"):
        assert out[k] > 0, k
    for k in ("sgemm", "reduce_weak", "scan_weak", "stencil", "spmv"):  # per-step hipEvent device time
        assert 0 < out[f"{k}_device_ms_min"] <= out[f"{k}_device_ms_median"] <= out[f"{k}_device_ms_max"], k
    assert out["stencil_bit_exact"] and out["stencil_finite"] and out["stencil_timed_grid_bit_exact"]
    assert out["scan_full_max_rel_err_vs_fp64"] < 1e-5 and out["scan_weak_lookback_ok"]
    assert out["sgemm_max_rel_err_vs_fp64"] < 1e-5 and out["spmv_max_rel_err_vs_fp64"] < 1e-5
    assert out["sgemm_fp32_via_bf16x6_tflops"] > 0 and out["sgemm_fp32_via_bf16x6_max_rel_err_vs_fp64"] < 1e-5
    assert out["reduce_strong_rel_err_vs_fp64"] < 1e-5 and out["scan_strong_rel_err_vs_fp64"] < 1e-5
    assert not [k for k in out if k.endswith("_error")], out


def test_bench_small_one_gpu(gpu):
    _check_line(_bench(1, "--steps", "2", "--warmup", "1", "--small", "--no-ref"), 1)


def _ngpu():
    return torch.cuda.device_count()


def test_bench_more_gpus_than_visible_is_refused(gpu):
    """`bench.py --gpus N` with N > the visible GPUs (no launcher): a clear error and a non-zero exit, no line."""
    n = _ngpu() + 1
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--small"], capture_output=True,
                       text=True, timeout=120, env=cli_env())
    assert r.returncode == 2 and f"--gpus {n} but only {n - 1} GPU(s) visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_wrong_result_fails_on_the_gpu(gpu):
    """A perturbed timed SGEMM C (one element; the old 8-row sample would have missed it) fails the full fp64 check:
    the line prints with sgemm_check_failed and the run exits 1."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--steps", "1", "--warmup", "0", "--size", "1024", "--no-ref",
           "--sections", "sgemm", "--inject-fault", "sgemm:0:perturb"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=cli_env())
    assert r.returncode == 1, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["sgemm_check_failed"] == ["sgemm_max_rel_err_vs_fp64"] and out["checks_passed"] is False


@pytest.mark.parametrize("nproc", [2, 4, 8])
def test_bench_ranks_share_one_gpu_over_gloo(gpu, nproc):
    """The whole N>1 bench path on ONE GPU: nproc torchrun ranks run their own GPU kernels (ghost-layout sliced
    SpMV with 2 exchange chunks, stencil slabs with the interior / two-span edge launches, seeded multi-rank scan,
    strong and weak reduce, weak SGEMM) while gloo carries the messages through host memory; every section's
    correctness check must pass (timings are meaningless: the ranks share the GPU)."""
    out = _bench(nproc, "--steps", "2", "--warmup", "1", "--no-ref", "--backend", "gloo", "--size", "2048",
                 "--reduce-n", "5e7", "--stencil-n", "2048", "--spmv-rows", "5e5", "--spmv-nnz", "5e6", timeout=110)
    _check_line(out, nproc)
    assert out["spmv_exchange"] == "ghost" and out["spmv_chunks"] == 2 and out["spmv_slices"] >= 16 and out["spmv_colsplit"]
    assert out["stencil_updates_per_step"] == 6  # auto_fuse of 1024 / 512 / 256-row slabs


@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 visible GPUs")
def test_bench_small_torchrun_all_gpus(gpu):
    n = min(_ngpu(), 8)
    _check_line(_bench(n, "--steps", "2", "--warmup", "1", "--small", "--no-ref"), n)


@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 visible GPUs")
def test_bench_self_launch_all_gpus_rccl(gpu):
    """The driver's own command shape: `python bench.py --gpus N` (no launcher) runs N RCCL ranks."""
    n = min(_ngpu(), 8)
    _check_line(_bench(n, "--steps", "2", "--warmup", "1", "--small", "--no-ref", self_launch=True), n)


def test_bench_self_launch_two_ranks_share_one_gpu(gpu):
    """`bench.py --gpus 2 --backend gloo` without a launcher: two ranks (sharing the GPU over gloo) in one line."""
    out = _bench(2, "--steps", "2", "--warmup", "1", "--no-ref", "--backend", "gloo", "--small", timeout=110,
                 self_launch=True)
    _check_line(out, 2)


@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 visible GPUs")
def test_region_torchrun_rccl_writes_golden(gpu, tmp_path):
    from parallel_c_programs_amd.parallel import free_port

    n = min(_ngpu(), 8)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "parallel_c_programs_amd.cli.run_region",
           str(ASSETS / "pic1.bmp")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=cli_env())
    assert r.returncode == 0, r.stderr[-3000:]
    assert np.array_equal(bmp.read(tmp_path / "out.bmp"), bmp.read(ASSETS / "region_pic1_golden.bmp"))


@pytest.mark.parametrize("parts", [1, 2, 3, 4])
def test_volume_zslabs_emulated_on_one_gpu(gpu, parts):
    """Every slab stage of a `parts`-rank z-slab decomposition on one GPU: the slab grower (halo planes as read-only
    seeds) and the pipelined slab caster reproduce the single-volume region and the f64 global caster bit for bit."""
    from parallel_c_programs_amd import ops
    from parallel_c_programs_amd.parallel import emulate_slabs

    vol = ops.create_volume(512, device=gpu, seed=0)
    reg_ref, _ = ops.region3d(vol)
    reg_ref = (reg_ref != 0).to(torch.uint8)
    img_ref = ops.raycast(vol, reg_ref, 64, method="global")
    reg, img, outer = emulate_slabs(512, parts, gpu, image_dim=64)
    assert int(reg.sum()) == 2197899 and torch.equal(reg, reg_ref)
    assert torch.equal(img, img_ref)
    assert outer == 1 if parts == 1 else outer >= 2


@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 visible GPUs")
def test_volume3d_torchrun_rccl(gpu, tmp_path):
    from parallel_c_programs_amd.parallel import free_port

    n = min(_ngpu(), 8)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "parallel_c_programs_amd.cli.run_volume3d",
           "--image-dim", "64"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=cli_env(), cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["region_voxels"] == 2197899 and out["image_sum"] == 127183


@pytest.mark.parametrize("nproc", [2, 4, 8])
def test_region_ranks_share_one_gpu_over_gloo(gpu, tmp_path, nproc):
    """The reference's MPI region-growing app at nproc ranks on ONE GPU (gloo carries scatter, halo exchanges,
    MAX termination and gather through host memory; every rank's grow kernels run on the GPU): out.bmp equals
    the reference's golden output."""
    from parallel_c_programs_amd.parallel import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "parallel_c_programs_amd.cli.run_region",
           str(ASSETS / "pic1.bmp"), "--backend", "gloo", "--device", "cuda", "--out", str(tmp_path / "out.bmp")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=cli_env())
    assert r.returncode == 0, r.stderr[-3000:]
    assert np.array_equal(bmp.read(tmp_path / "out.bmp"), bmp.read(ASSETS / "region_pic1_golden.bmp"))


@pytest.mark.parametrize("nproc", [2, 4])
def test_volume3d_ranks_share_one_gpu_over_gloo(gpu, tmp_path, nproc):
    """The z-slab 3-D pipeline (slab generation, tiled slab growing with halo planes and device MAX termination,
    pipelined slab ray caster) at nproc ranks on ONE GPU over gloo: the reference box region and image."""
    from parallel_c_programs_amd.parallel import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "parallel_c_programs_amd.cli.run_volume3d",
           "--image-dim", "64", "--backend", "gloo", "--device", "cuda"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=cli_env(), cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["region_voxels"] == 2197899 and out["image_sum"] == 127183


@pytest.mark.parametrize("world,fuse,m", [(2, 6, 1), (8, 6, 1), (8, 4, 1), (4, 8, 1), (8, 6, 2), (4, 8, 2), (8, 4, 3)])
def test_stencil_slabs_emulated_on_one_gpu(gpu, world, fuse, m):
    """Every rank of a `world`-rank row-slab stencil on one GPU: halos copied slab to slab (what the grouped RCCL
    send/recv moves), then StencilSlab.step's overlapped path itself (interior rows, then both boundary bands in
    one two-span launch) — bit-identical to the single-domain oracle. At
    world 8 a slab of a 2048-row grid is a short range, so this runs the v2 kernel's 24-rows-per-wave launch with
    interior and edge waves. m > 1: the deep-halo schedule (edge spans reaching into the halo, extended full launches
    at the later phases)."""
    from parallel_c_programs_amd.parallel.dist import Context
    from parallel_c_programs_amd.parallel.stencil import StencilSlab, reference_run

    class Emulated(Context):  # a rank of a distributed run whose halo exchange the test performs itself
        @property
        def distributed(self):
            return True

    n, cols, steps = 2048, 1000, 2 * m * fuse + fuse  # (m > 1: two deep-halo periods and one exchange step)
    slabs = [StencilSlab(Emulated(rank=r, world=world, device=gpu), n, cols, fuse=fuse, halo_mult=m)
             for r in range(world)]
    for s in slabs:
        s._post_exchange = lambda: []
    for _ in range(steps // fuse):
        for r, s in enumerate(slabs):  # halo exchange at the period's first step: m * T rows from each neighbour
            if s.phase:
                continue
            h = s.halo
            if r > 0:
                s.u[0:h].copy_(slabs[r - 1].u[slabs[r - 1].rows:slabs[r - 1].rows + h])
            if r < world - 1:
                s.u[s.rows + h:s.rows + 2 * h].copy_(slabs[r + 1].u[h:2 * h])
        for s in slabs:
            s.step(overlap=True)
    got = torch.cat([s.interior() for s in slabs]).cpu()
    ref = reference_run(n, steps, cols, device=gpu).cpu()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))


@pytest.mark.parametrize("world", [2, 8])
def test_spmv_colsplit_phases_emulated_on_one_gpu(gpu, world):
    """The column-split product of one rank (SlicedCSR cut at the first layout column of chunk 1): the products of the
    slices below the split, then of the others, then the combine — bit-identical to the one-call product of the same
    matrix (same partials, same slice-order combine) and within 1e-5 of fp64; and the two row chunks' chunk-0-column
    products as one paired launch (same bits)."""
    from parallel_c_programs_amd.parallel.dist import Context
    from parallel_c_programs_amd.parallel.spmv import DistributedSpMV

    for r in sorted({0, world - 1}):
        d = DistributedSpMV.powerlaw(Context(rank=r, world=world, device=gpu), 300_000, 3_000_000, slices=16, chunks=2,
                                     colsplit=True)
        assert d.colsplit and d.slices == 16 and 0 < d.col_split < d.n_pad
        xp = torch.rand(d.n_pad, device=gpu)
        for c, (a, b, part) in enumerate(d.parts):
            if b <= a:
                continue
            assert part.col_split == d.col_split and int(part.bounds[7]) == d.col_split
            full = part.spmv(xp)
            dst = torch.full_like(full, float("nan"))
            part.product_phase(xp, 0, c)
            part.product_phase(xp, 1, c, dst)
            assert torch.equal(dst, full), (r, c)
            ref = part.reference(xp)
            assert ((dst.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5
        # both row chunks' chunk-0-column products as ONE paired launch (the production column-split step): each
        # chunk's combine then gives the same bits
        (a0, b0, p0), (a1, b1, p1) = d.parts
        if b0 > a0 and b1 > a1:
            full0, full1 = p0.spmv(xp), p1.spmv(xp)
            p0.products_pair(p1, xp, (0, p0.n_slices // 16), (0, p1.n_slices // 16))
            y0, y1 = torch.full_like(full0, float("nan")), torch.full_like(full1, float("nan"))
            p0.product_phase(xp, 1, 0, y0)
            p1.product_phase(xp, 1, 1, y1)
            assert torch.equal(y0, full0) and torch.equal(y1, full1), r


@pytest.mark.parametrize("exchange", ["ghost", "allgather"])
@pytest.mark.parametrize("world", [2, 8])
def test_spmv_ranks_emulated_on_one_gpu(gpu, world, exchange):
    """Every rank's local product of the distributed power-law SpMV on one GPU: nnz-balanced row blocks, columns
    renumbered into the compact ghost layout or the padded all-gather layout, 4 pipeline chunks per rank,
    XCD-sliced compact-partial kernel — each chunk checked against the fp64 product of the same rows."""
    from parallel_c_programs_amd.parallel.dist import Context
    from parallel_c_programs_amd.parallel.spmv import DistributedSpMV

    for r in sorted({0, world // 2, world - 1}):
        d = DistributedSpMV.powerlaw(Context(rank=r, world=world, device=gpu), 300_000, 3_000_000, slices=16, chunks=4,
                                     exchange=exchange)
        assert d.chunks == 4 and (d.n_pad >= d.n if exchange == "allgather" else d.rows < d.n_pad < d.n)
        xp = torch.rand(d.n_pad, device=gpu)
        got = []
        for c, (a, b, part) in enumerate(d.parts):
            if b > a:
                dst = torch.empty(b - a, device=gpu)
                d._mul(part, xp, dst)
                got.append(dst.double())
        got = torch.cat(got)
        ref = d.reference_local(xp)
        assert got.shape == ref.shape == (d.rows,)
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-5, (r, err)


_NEIGHBOUR_SCRIPT = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["PCMX_ROOT"])
from parallel_c_programs_amd.parallel.dist import init, finalize
os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1")
ctx = init()
if not dist.is_initialized():  # world 1: init() leaves the group out; the call shapes still need one
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=ctx.device)
ctx.backend, ctx.world = "nccl", 1
dev = ctx.device
a = torch.arange(12, dtype=torch.float32, device=dev).view(3, 4)
b = torch.zeros(3, 4, device=dev)
class Ctx(type(ctx)):
    @property
    def distributed(self):
        return True
c = Ctx(0, 1, 0, dev, "nccl")
for w in c.neighbour_exchange([(0, a[1], b[2])], async_op=True):
    w.wait()
c.neighbour_exchange([(0, a[0:2].reshape(-1), b[0:2].reshape(-1))])
e = a.new_empty(0)
dist.all_to_all([e], [e])  # zero-size entries (non-neighbours) pass through RCCL's grouped send/recv
torch.cuda.synchronize()
assert torch.equal(b[2], a[1]) and torch.equal(b[0:2], a[0:2]), b
c.neighbour_exchange([])  # a rank without neighbours still enters the collective
print("neighbour_exchange ok")
# the RCCL call shapes the N > 1 bench paths use, on the same world-1 group:
# all_to_all_single with explicit split lists (one of them zero) ...
src = torch.arange(5, dtype=torch.float32, device=dev)
dst = torch.zeros(5, device=dev)
dist.all_to_all_single(dst, src, [5], [5])
z = torch.zeros(0, device=dev)
dist.all_to_all_single(z, z, [0], [0])
assert torch.equal(dst, src)
# ... all_gather_into_tensor into a slice of a bigger tensor (allgather SpMV layout, global_scan totals) ...
big = torch.zeros(10, device=dev)
dist.all_gather_into_tensor(big[3:7], src[1:5])
assert torch.equal(big[3:7], src[1:5]) and float(big.sum()) == float(src[1:5].sum())
# ... Context.exchange with per-peer views (the ghost exchange) ...
out = torch.zeros(6, device=dev)
c.exchange([out[2:5]], [src[0:3]])
torch.cuda.synchronize()
assert torch.equal(out[2:5], src[0:3]) and float(out[0:2].sum()) == 0 and float(out[5]) == 0
print("rccl call shapes ok")
# the native grouped exchange (dedicated RCCL communicator, csrc/comm/exchange_rccl.hip): probed at creation, then
# segments to / from every rank (here: itself) through Context.exchange_segments, an out-of-bounds segment refused
from parallel_c_programs_amd.parallel.dist import native_exchange, native_exchange_active
nx = native_exchange(c)
assert nx is not None and native_exchange_active(c)
snd = torch.arange(10, dtype=torch.float32, device=dev) + 1
rcv = torch.zeros(16, device=dev)
for w in c.exchange_segments(3, snd, [2], [5], rcv, [9], [5]):
    w.wait()
torch.cuda.synchronize()
assert torch.equal(rcv[9:14], snd[2:7]) and float(rcv[:9].sum()) == 0 and float(rcv[14:].sum()) == 0, rcv
try:
    c.exchange_segments(3, snd, [8], [5], rcv, [0], [5])
    raise SystemExit("out-of-bounds send segment accepted")
except RuntimeError:
    pass
assert nx.healthy()
print("native exchange ok")
# ... and the distributed SpMV step (ghost layout set-up exchange, _post_chunk per chunk, step_padded) and the
# seeded global scan, through a context that takes the N > 1 branches
from parallel_c_programs_amd.parallel.spmv import DistributedSpMV
from parallel_c_programs_amd.parallel.collectives import global_scan
d = DistributedSpMV.powerlaw(c, 200_000, 2_000_000, slices=16, chunks=3)
assert d.chunks == 3 and c.distributed
xp = torch.rand(d.n_pad, device=dev)
for k in range(d.chunks):
    for w in d._post_chunk(torch.zeros(d.n_pad, device=dev), k):
        w.wait()
y = d.step_padded(xp)
err = d.layout_max_rel_err(y, xp)
assert err < 1e-5, err
x = torch.rand(100_000, device=dev)
ys = global_scan(x, c)
assert torch.allclose(ys.double(), torch.cumsum(x.double(), 0), rtol=1e-5, atol=1e-2)
print("distributed spmv/scan branches ok", err)
# the column-split pipeline as an iteration on RCCL's own stream ordering (world 1: the list all_to_all moves nothing,
# but every work.wait() / stream dependency of the deferred schedule is RCCL's)
d2 = DistributedSpMV.powerlaw(c, 200_000, 2_000_000, slices=16, chunks=2, colsplit=True)
assert d2.colsplit
xp2 = torch.rand(d2.n_pad, device=dev)
a = d2.iterate(xp2, 5, defer=True).clone()
b = d2.iterate(xp2, 5, defer=False)
assert torch.equal(a, b)
err2 = d2.iterate_max_rel_err(xp2, 5)
assert err2 < 1e-5, err2
print("deferred spmv pipeline on rccl ok", err2)
dist.destroy_process_group()
"""

_NATIVE_FALLBACK_SCRIPT = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["PCMX_ROOT"])
from parallel_c_programs_amd.parallel.dist import init, native_exchange, native_exchange_active
os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", PCMX_XCOMM_FAIL_RANK="0")
ctx = init()
if not dist.is_initialized():
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=ctx.device)
ctx.backend, ctx.world = "nccl", 1
dev = ctx.device
class Ctx(type(ctx)):
    @property
    def distributed(self):
        return True
c = Ctx(0, 1, 0, dev, "nccl")
# a rank that reports a failed probe sends the job to the torch path (the communicator closed, no exception)
assert native_exchange(c) is None and not native_exchange_active(c)
snd = torch.arange(10, dtype=torch.float32, device=dev) + 1
rcv = torch.zeros(16, device=dev)
for w in c.exchange_segments(3, snd, [2], [5], rcv, [9], [5]):
    w.wait()
torch.cuda.synchronize()
assert torch.equal(rcv[9:14], snd[2:7]), rcv
print("native fallback ok")
dist.destroy_process_group()
"""

_ITERATE_SCRIPT = r"""
import os, sys, torch
sys.path.insert(0, os.environ["PCMX_ROOT"])
from parallel_c_programs_amd.parallel.dist import init, finalize, LazyContext
from parallel_c_programs_amd.parallel.spmv import DistributedSpMV
ctx = init(backend="gloo", device="cuda")
c = LazyContext.of(ctx)  # exchanges land only when waited for
d = DistributedSpMV.powerlaw(c, 300_000, 3_000_000, slices=16, chunks=2, colsplit=True)
assert d.colsplit and d.sliced
g = torch.Generator(device=ctx.device).manual_seed(3)
xp = d.to_padded(torch.rand(d.n, device=ctx.device, generator=g))
a = d.iterate(xp, 5, defer=True).clone()
b = d.iterate(xp, 5, defer=False)
same = ctx.max_over_ranks(0.0 if torch.equal(a, b) else 1.0) == 0.0
err = d.iterate_max_rel_err(xp, 5, defer=True)
if ctx.rank == 0:
    print("ITER", same, err, flush=True)
finalize(ctx)
"""


def test_neighbour_exchange_rccl_call_shape(gpu, tmp_path):
    """The RCCL-only branches of the N > 1 paths on a world-1 NCCL group (RCCL refuses two ranks on one GPU, and
    the gloo GPU tests take the host-staged branch): Context.exchange / neighbour_exchange (one list all_to_all,
    zero-size entries for non-neighbours, the rank as its own neighbour, a rank with no neighbours),
    all_to_all_single with split lists incl. zero, all_gather_into_tensor into a slice, and DistributedSpMV's
    ghost set-up + _post_chunk + step_padded and the seeded global_scan through a context that takes the
    distributed branches."""
    from parallel_c_programs_amd.parallel import free_port

    script = tmp_path / "nb.py"
    script.write_text(_NEIGHBOUR_SCRIPT)
    env = dict(cli_env(), PCMX_ROOT=str(ROOT), MASTER_PORT=str(free_port()))
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "neighbour_exchange ok" in r.stdout, r.stderr[-3000:]
    assert "rccl call shapes ok" in r.stdout and "distributed spmv/scan branches ok" in r.stdout, r.stderr[-3000:]
    assert "deferred spmv pipeline on rccl ok" in r.stdout, r.stderr[-3000:]
    assert "native exchange ok" in r.stdout, r.stderr[-3000:]


def test_native_exchange_probe_failure_falls_back(gpu, tmp_path):
    """A rank whose native-exchange probe fails (test hook PCMX_XCOMM_FAIL_RANK) makes the job agree on the torch
    path: native_exchange() returns None, the dedicated communicator is closed, and exchanges still deliver."""
    from parallel_c_programs_amd.parallel import free_port

    script = tmp_path / "fallback.py"
    script.write_text(_NATIVE_FALLBACK_SCRIPT)
    env = dict(cli_env(), PCMX_ROOT=str(ROOT), MASTER_PORT=str(free_port()))
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "native fallback ok" in r.stdout, r.stderr[-3000:]


@pytest.mark.parametrize("world", [2, 4])
def test_spmv_deferred_pipeline_iterates_ranks_share_one_gpu(gpu, tmp_path, world):
    """The steady-state column-split pipeline as an ITERATION on the GPU kernels (sliced phase launches): `world`
    ranks share the GPU over gloo through LazyContext (an exchange lands only when waited for), 5 chained steps
    x <- A x with each step's chunk-1 exchange in flight into the next: bit-identical to the same steps with every
    exchange finished in its step, and within 1e-5 of fp64 A^5 x on every layout entry."""
    from parallel_c_programs_amd.parallel import free_port

    script = tmp_path / "it.py"
    script.write_text(_ITERATE_SCRIPT)
    env = dict(cli_env(), PCMX_ROOT=str(ROOT))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), str(script)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("ITER")][0].split()
    assert line[1] == "True" and float(line[2]) < 1e-5, line
