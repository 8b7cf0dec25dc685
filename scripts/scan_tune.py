"""Scan schedule A/B on 1e9 f32 (pcmx_scan_f32_variant through ctypes): 0 persistent R16xW8, 1 persistent R8xW16,
2 parked-tile R16xW8, 3 parked-tile R8xW16, 4 parked-tile R16xW8 + early polls (production), 5 = 4 with the next tile's loads issued before the scan
(round 6), 6 = the same loads issued after wave 0's early polls, 7 / 8 = 4 / 6 with
branch-free buffer-descriptor tile loads. Device time, GB/s
(8 B/element), error vs fp64. Before timing, every variant is checked on ragged sizes, exclusive mode, an init
offset and in place.
usage: python scripts/scan_tune.py [n] [variants, comma separated] [rounds]"""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd._native import hip_lib  # noqa: E402
from parallel_c_programs_amd.utils.timing import device_time_ms  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**9
variants = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 2]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
lib = hip_lib()
lib.pcmx_scan_workspace_bytes.restype = ctypes.c_longlong
stream = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731


def scan(x, y, ws, variant, exclusive=0, init=None, verify=True):
    rc = lib.pcmx_scan_f32_variant(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                   ctypes.c_longlong(x.numel()), exclusive,
                                   ctypes.c_void_p(init.data_ptr()) if init is not None else None,
                                   ctypes.c_void_p(ws.data_ptr()), None, variant, stream())
    assert rc == 0, rc
    if not verify:
        return
    rc = lib.pcmx_scan_check(ctypes.c_void_p(ws.data_ptr()), stream())
    assert rc == 0, f"look-back timeout rc={rc}"


def check(variant):
    for m in (1, 5, 32768, 32769, 300_001, 32768 * 700 + 13):
        x = torch.randint(-8, 9, (m,), device="cuda").float()  # small integers: every prefix is exact in f32
        ws = torch.empty(lib.pcmx_scan_workspace_bytes(ctypes.c_longlong(m)), dtype=torch.uint8, device="cuda")
        init = torch.tensor([3.0], device="cuda")
        ref = torch.cumsum(x.double(), 0) + 3.0
        for exclusive in (0, 1):
            y = torch.full_like(x, float("nan"))
            scan(x, y, ws, variant, exclusive, init)
            want = ref if not exclusive else torch.cat([torch.tensor([3.0], device="cuda", dtype=torch.float64),
                                                        ref[:-1]])
            assert torch.equal(y.double(), want), (variant, m, exclusive)
        z = x.clone()
        scan(z, z, ws, variant)  # in place
        assert torch.equal(z.double(), ref - 3.0), (variant, m, "in-place")
    print(f"variant {variant}: ragged / exclusive / init / in-place exact", flush=True)


for v in variants:
    check(v)
x = torch.empty(n, device="cuda")
ops.rand_uniform_(x, 7, 0.0, 1.0)
y = torch.empty_like(x)
ws = torch.empty(lib.pcmx_scan_workspace_bytes(ctypes.c_longlong(n)), dtype=torch.uint8, device="cuda")
ref = torch.cumsum(x[: 1 << 22].double(), 0)
tail_ref = x.double().sum().item()
for _ in range(rounds):
    for v in variants:
        ms = device_time_ms(lambda: scan(x, y, ws, v, verify=False), reps=10, warmup=2)
        scan(x, y, ws, v)  # one more, checked for a look-back timeout
        err = ((y[: 1 << 22].double() - ref).abs().max() / ref[-1]).item()
        tail = abs(y[-1].item() - tail_ref) / tail_ref
        print(f"variant={v}  {ms:7.3f} ms  {8 * n / ms / 1e6:7.1f} GB/s  rel_err={err:.2e}  tail_rel={tail:.2e}",
              flush=True)
