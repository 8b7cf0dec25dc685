"""Failure surfacing: conditions that used to yield a silently wrong or incomplete result must raise.

  * scan: a decoupled look-back that gives up (stalled predecessor) marks the result invalid. Forced with the
    test-only fault-injection build of scan.hip (libpcmx_faultinj.so, -DPCMX_FAULT_INJECT: tile 1 never sees
    its predecessor and exhausts a 64-poll spin limit).
  * region growing: a fixpoint loop that runs out of max_launches with work left returns
    PCMX_ERR_NOT_CONVERGED (-2), which the torch ops raise.
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
