"""Device introspection (replaces print_properties, ref 5-cuda-region-growing/raycast.cu:99-110, and the
OpenCL printPlatformInfo/printDeviceInfo, ref 6-opencl-region-growing/clutil.c:63-122)."""
from __future__ import annotations

import torch


def print_device_info(device: int = 0) -> None:
    """Prints device count, name, gfx arch, CUs, LDS, L2, HBM size and clocks (native HIP query)."""
    if torch.cuda.is_available():
        from .._native import ops

        ops().device_info(device)
        return
    print("Device count: 0")
    print("(no HIP device visible; host path only)")


def device_summary(device: int = 0) -> dict:
    if not torch.cuda.is_available():
        return {"device_count": 0}
    p = torch.cuda.get_device_properties(device)
    return {
        "device_count": torch.cuda.device_count(),
        "name": p.name,
        "arch": getattr(p, "gcnArchName", ""),
        "compute_units": p.multi_processor_count,
        "total_memory_gib": round(p.total_memory / 2**30, 1),
    }
