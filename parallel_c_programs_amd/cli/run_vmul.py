"""Vector multiply demo (ref 6-opencl-region-growing/multiply_opencl.c + multiply_opencl.cl): 1024 elements,
a[i] = i + 1, b[i] = 1 / (i + 1) (so every product is 1), prints the device info then the
"Host\\tDevice" table of the first 10 results ("%0.2f\\t%0.2f")."""
from __future__ import annotations

import argparse

import torch

from .. import ops
from ..utils.device import print_device_info

SIZE = 1024


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="run_vmul")
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    dev = torch.device(a.device or ("cuda" if torch.cuda.is_available() else "cpu"))
    i = torch.arange(SIZE, dtype=torch.float32)
    x, y = i + 1, 1.0 / (i + 1)
    host = x * y
    if dev.type == "cuda":
        print_device_info(dev.index or 0)
    dev_r = ops.vmul(x.to(dev), y.to(dev)).cpu()
    print("Host\tDevice")
    for k in range(10):
        print(f"{host[k].item():0.2f}\t{dev_r[k].item():0.2f}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
