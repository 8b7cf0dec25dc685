"""Failure surfacing: conditions that used to yield a silently wrong or incomplete result must raise.

  * scan: a decoupled look-back that gives up (stalled predecessor) marks the result invalid. Forced with the
    test-only fault-injection build of scan.hip (libpcmx_faultinj.so, -DPCMX_FAULT_INJECT: tile 1 never sees
    its predecessor and exhausts a 64-poll spin limit).
  * region growing: a fixpoint loop that runs out of max_launches with work left returns
    PCMX_ERR_NOT_CONVERGED (-2), which the torch ops raise.
  * the bench's stencil check: a one-lane neighbour swap in the fused kernel (the same fault-injection build of
    stencil.hip) must fail the timed-grid check on the bench's random grid.
"""
import ctypes

import pytest
import torch
from conftest import ROOT

from parallel_c_programs_amd import ops
from parallel_c_programs_amd._native import ops as native

pytestmark = pytest.mark.gpu

PCMX_ERR_NOT_CONVERGED, PCMX_ERR_TIMEOUT = -2, -3


def _faultinj():
    path = ROOT / "parallel_c_programs_amd" / "lib" / "libpcmx_faultinj.so"
    assert path.exists(), "build() must produce the test-only fault-injection library"
    lib = ctypes.CDLL(str(path))
    lib.pcmx_scan_workspace_bytes.restype = ctypes.c_longlong
    lib.pcmx_scan_workspace_bytes.argtypes = [ctypes.c_longlong]
    lib.pcmx_scan_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.pcmx_scan_check.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.pcmx_stencil5xT_bf16_spans_shape.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 9 + [
        ctypes.c_longlong, ctypes.c_longlong, ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
    return lib


def test_scan_lookback_timeout_is_reported(gpu):
    lib = _faultinj()
    n = 5 * 32768 + 17  # several 128-KiB tiles; tile 1's look-back is forced to stall
    x = torch.rand(n, device=gpu)
    y = torch.empty_like(x)
    ws = torch.zeros(lib.pcmx_scan_workspace_bytes(n), dtype=torch.uint8, device=gpu)
    err = torch.zeros(1, dtype=torch.int32, device=gpu)
    stream = ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)
    rc = lib.pcmx_scan_f32(x.data_ptr(), y.data_ptr(), n, 0, None, ws.data_ptr(), err.data_ptr(), stream)
    assert rc == 0  # the launch itself is fine ...
    torch.cuda.synchronize()
    assert int(err.item()) == 1  # ... but the sticky error word says the result is invalid
    assert lib.pcmx_scan_check(ws.data_ptr(), stream) == PCMX_ERR_TIMEOUT


def test_production_scan_reports_no_timeout(gpu):
    x = torch.rand(3 * 32768 + 5, device=gpu)
    y = ops.scan(x)
    native().scan_check(0)  # raises if any scan on device 0 gave up a look-back
    assert torch.allclose(y.double(), torch.cumsum(x.double(), 0), rtol=1e-5, atol=1e-3)


def _serpentine(n: int) -> torch.Tensor:
    """Padded (n+2)^2 maze: walls every 4th row with the gap alternating between the ends, so the corner seed's
    4-connected region is one long serpentine path (many launches to converge)."""
    img = torch.zeros(n + 2, n + 2, dtype=torch.uint8)
    for k, r in enumerate(range(4, n, 4)):
        img[r, 1:n + 1] = 200
        gap = 2 if k % 2 else n - 1
        img[r, gap] = 0
    return img


def test_region2d_not_converged_raises(gpu):
    img = _serpentine(1024).to(gpu)
    reg = torch.zeros_like(img)
    reg[1, 1] = 1
    with pytest.raises(RuntimeError, match="not converged"):
        ops.region2d_grow_padded_(reg, img, 2, batch=1, max_launches=1)
    # with launches to spare the same call converges, and the region follows the whole serpentine
    reg2 = torch.zeros_like(img)
    reg2[1, 1] = 1
    launches = ops.region2d_grow_padded_(reg2, img, 2)
    assert launches > 1
    interior = reg2[1:-1, 1:-1]
    assert int(interior.sum()) == int((img[1:-1, 1:-1] == 0).sum())


@pytest.mark.parametrize("tiled", [True, False])
def test_region3d_not_converged_raises(gpu, tiled):
    data = ops.create_volume(128, device=gpu, seed=0)
    data.zero_()  # one uniform volume: the whole cube is the region, many BFS levels from a corner seed
    reg = torch.zeros_like(data)
    reg[0, 0, 0] = 2 if not tiled else 1
    with pytest.raises(RuntimeError, match="not converged"):
        native().region3d_grow_(reg, data, 1, tiled, 1, 1)


def _faulty_fused_step(lib):
    """ops.stencil5_fused_step_ on the fault-injection build's kernel (lane 17 swaps a neighbour)."""
    def fused(u, out, global_row0=0, global_rows=None, k=0.2, halo=1, steps=2, row_range=None, shape=0):
        rows, cols = u.shape[0] - 2 * halo, u.shape[1]
        global_rows = rows if global_rows is None else global_rows
        r0, r1 = row_range or (0, rows)
        stream = ctypes.c_void_p(torch.cuda.current_stream(u.device).cuda_stream)
        rc = lib.pcmx_stencil5xT_bf16_spans_shape(u.data_ptr(), out.data_ptr(), rows, cols, cols, halo, steps, r0, r1,
                                                  0, 0, global_row0, global_rows, k, shape, stream)
        assert rc == 0
        return out
    return fused


def test_stencil_check_catches_one_lane_neighbour_swap(gpu, monkeypatch):
    """The bench's stencil check (workloads.Stencil.check: the timed grid bit for bit against plain-PyTorch single
    steps) on its random grid: it passes on the production kernel and FAILS when one lane of every strip reads its
    east neighbour as its west one (fault-injection build), a bug a constant grid region would hide."""
    from parallel_c_programs_amd.models import workloads as W
    from parallel_c_programs_amd.parallel import stencil as PS
    from parallel_c_programs_amd.parallel.dist import Context

    lib = _faultinj()
    ctx = Context(device=gpu)
    good = W.Stencil(ctx, n=2048, fuse=8)
    for _ in range(3):
        good.step()
    assert good.check()["check_passed"]
    monkeypatch.setattr(PS, "stencil5_fused_step_", _faulty_fused_step(lib))
    bad = W.Stencil(ctx, n=2048, fuse=8)
    for _ in range(3):
        bad.step()
    c = bad.check()
    assert not c["timed_grid_bit_exact"] and not c["check_passed"]
