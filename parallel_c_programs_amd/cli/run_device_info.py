"""Device properties (ref print_properties, 5-cuda-region-growing/raycast.cu:99-110; OpenCL
printPlatformInfo/printDeviceInfo, 6-opencl-region-growing/clutil.c:63-122)."""
from __future__ import annotations

from ..utils.device import print_device_info


def main(argv=None) -> int:
    import torch

    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    if n == 0:
        print_device_info(0)
    for d in range(n):
        print_device_info(d)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
