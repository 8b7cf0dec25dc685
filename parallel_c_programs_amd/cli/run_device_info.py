"""Device properties (ref print_properties, 5-cuda-region-growing/raycast.cu:99-110; OpenCL
printPlatformInfo/printDeviceInfo, 6-opencl-region-growing/clutil.c:63-122).

Default: the reference-style property listing of every visible device (native HIP query). Beyond it:
  --json           one JSON object: per-device summary (name, gfx arch, CUs, HBM) and the peer-access matrix (which
                   device pairs can address each other's memory over xGMI)
  --require-arch A exit 1 unless every device is arch A (e.g. gfx950, the only target the kernels are built for)
  --probe          quick per-device measurements with this package's kernels: HBM read (reduce over 1 GiB), HBM
                   write (fill of 1 GiB), f32 MFMA GEMM 4096^3, and with >= 2 devices the device-0 -> device-d copy
                   rate of 256 MiB (one xGMI path per pair) — a node sanity check before a multi-GPU run
"""
from __future__ import annotations

import argparse
import json

from ..utils.device import device_summary, print_device_info


def _peer_matrix(n: int) -> list[list[bool]]:
    import torch

    return [[i == j or torch.cuda.can_device_access_peer(i, j) for j in range(n)] for i in range(n)]


def _time_ms(fn, reps: int) -> float:
    import torch

    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def probe(device: int, n_dev: int, reps: int = 10) -> dict:
    """HBM read / write rate and f32 GEMM rate of one device; device 0 also times a copy to every other device."""
    import torch

    from .. import ops

    dev = torch.device("cuda", device)
    out = {"device": device}
    with torch.cuda.device(dev):
        x = torch.empty(1 << 28, device=dev)  # 1 GiB of f32
        ops.fill_(x, 1.0)
        ms = _time_ms(lambda: ops.reduce(x, "sum"), reps)
        out["hbm_read_gbps"] = round(x.numel() * 4 / ms / 1e6, 1)
        ms = _time_ms(lambda: ops.fill_(x, 2.0), reps)
        out["hbm_write_gbps"] = round(x.numel() * 4 / ms / 1e6, 1)
        del x
        a = torch.rand(4096, 4096, device=dev)
        b = torch.rand(4096, 4096, device=dev)
        ms = _time_ms(lambda: ops.sgemm(a, b), reps)
        out["sgemm_4096_tflops"] = round(2 * 4096 ** 3 / ms / 1e9, 1)
        del a, b
        if device == 0 and n_dev > 1:
            src = torch.empty(1 << 26, device=dev)  # 256 MiB
            out["copy_to_peer_gbps"] = {}
            for d in range(1, n_dev):
                dst = torch.empty(1 << 26, device=torch.device("cuda", d))
                ms = _time_ms(lambda: dst.copy_(src, non_blocking=True), reps)
                out["copy_to_peer_gbps"][d] = round(src.numel() * 4 / ms / 1e6, 1)
                del dst
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="run_device_info")
    ap.add_argument("--json", action="store_true", help="summary + peer-access matrix as one JSON object")
    ap.add_argument("--require-arch", default=None, metavar="ARCH", help="exit 1 unless every device is ARCH")
    ap.add_argument("--probe", action="store_true", help="quick HBM / GEMM / peer-copy measurements (GPU)")
    a = ap.parse_args(argv)
    import torch

    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    if not (a.json or a.probe):
        if n == 0:
            print_device_info(0)
        for d in range(n):
            print_device_info(d)
    devices = [device_summary(d) for d in range(n)]
    if a.json:
        print(json.dumps({"device_count": n, "devices": devices, "peer_access": _peer_matrix(n) if n else []}),
              flush=True)
    if a.probe:
        if n == 0:
            print("run_device_info: --probe needs a GPU", flush=True)
            return 1
        for d in range(n):
            print(json.dumps(probe(d, n)), flush=True)
    if a.require_arch is not None:
        bad = [d for d in devices if not str(d.get("arch", "")).startswith(a.require_arch)]
        if n == 0 or bad:
            print(f"run_device_info: not every device is {a.require_arch}: "
                  f"{[d.get('arch') for d in devices] or 'no device'}", flush=True)
            return 1
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
