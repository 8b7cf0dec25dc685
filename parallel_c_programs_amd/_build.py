"""In-tree native build of every pcmx component (no JIT cache, nothing installed).

Artefacts (all git-ignored, all shipped to the GPU box by gpurun's snapshot):
  parallel_c_programs_amd/lib/libpcmx_cpu.so   host C library: BMP, matrix_t, SpMV, histogram, oracles
  parallel_c_programs_amd/lib/libpcmx_hip.so   HIP kernels for gfx950 + C-ABI launchers + device runtime
  parallel_c_programs_amd/_C.so                torch op registrations (TORCH_LIBRARY(pcmx, ...))
  bin/<tool>                                   reference-style CLIs (spmv, histogram_*, matrix_demo, ...)
  parallel_c_programs_amd/lib/libpcmx_faultinj.so  TEST ONLY: kernels built with -DPCMX_FAULT_INJECT (a forced
                                               scan look-back stall, a one-lane stencil neighbour swap) so tests can
                                               observe the error paths and the power of the checks

Everything is compiled for gfx950 only (`--offload-arch=gfx950`). Native libraries link the HIP runtime
that ships inside torch (torch/lib/libamdhip64.so, same SONAME as /opt/rocm's) with an rpath to it, so a
process never loads two HIP runtimes.

Usage: python -m parallel_c_programs_amd._build [--force] [--jobs N] [--only cpu|hip|torch|bin]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shlex
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = ROOT / "csrc"
LIB = PKG / "lib"
BIN = ROOT / "bin"
OBJ = ROOT / "build" / "obj"
ARCH = os.environ.get("PCMX_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")


def _torch_paths():
    import torch  # noqa: F401  (only needed for include/lib paths)
    from torch.utils import cpp_extension

    tdir = Path(torch.__file__).resolve().parent
    return [str(p) for p in cpp_extension.include_paths()], str(tdir / "lib"), torch


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _headers():
    return [p for p in (CSRC / "include").glob("*.h*")] + [p for p in CSRC.rglob("*.cuh")] + \
        [p for p in (CSRC / "kernels").glob("*.h")] + [p for p in (CSRC / "runtime").glob("*.h")]


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}):\n{' '.join(shlex.quote(c) for c in cmd)}\n{r.stdout}")
    return r.stdout


CPU_SRCS = ["cpu/bmp.c", "cpu/matrix.c", "cpu/spmv.c", "cpu/histogram.c", "cpu/vec.c", "cpu/oracles.c",
            "cpu/pipeline3d_host.c", "cpu/demos.c", "comm/comm_tcp.c", "comm/region_dist.c"]
CFLAGS = ["-O3", "-fPIC", "-std=gnu11", "-fopenmp", "-march=x86-64-v3", "-Wall", "-Wno-unknown-pragmas",
          f"-I{CSRC / 'include'}"]
# files whose float rounding must match the reference build bit-for-bit
NO_CONTRACT = {"cpu/oracles.c", "cpu/histogram.c", "cpu/spmv.c"}


def build_cpu(force=False, jobs=8):
    LIB.mkdir(parents=True, exist_ok=True)
    (OBJ / "cpu").mkdir(parents=True, exist_ok=True)
    hdrs = _headers()
    objs, todo = [], []
    for s in CPU_SRCS:
        src = CSRC / s
        o = OBJ / (s.replace("/", "_") + ".o")
        objs.append(o)
        flags = CFLAGS + (["-ffp-contract=off"] if s in NO_CONTRACT else [])
        if force or _newer(o, [src, *hdrs]):
            todo.append(["gcc", *flags, "-c", str(src), "-o", str(o)])
    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, todo))
    so = LIB / "libpcmx_cpu.so"
    if force or todo or not so.exists():
        _run(["gcc", "-shared", "-fopenmp", "-o", str(so), *map(str, objs), "-lm", "-lpthread"])
    return so


HIP_SRCS = sorted(str(p.relative_to(CSRC)) for p in (CSRC / "kernels").glob("*.hip")) + \
    sorted(str(p.relative_to(CSRC)) for p in (CSRC / "runtime").glob("*.hip")) + \
    sorted(str(p.relative_to(CSRC)) for p in (CSRC / "comm").glob("*.hip"))
HIPFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
            f"-I{CSRC / 'include'}", f"-I{CSRC / 'kernels'}", f"-I{CSRC / 'runtime'}",
            "-Wno-unused-result", "-Wno-pass-failed"]


def build_hip(force=False, jobs=8):
    _, tlib, _ = _torch_paths()
    LIB.mkdir(parents=True, exist_ok=True)
    (OBJ / "hip").mkdir(parents=True, exist_ok=True)
    hdrs = _headers()
    objs, todo = [], []
    for s in HIP_SRCS:
        src = CSRC / s
        o = OBJ / (s.replace("/", "_") + ".o")
        objs.append(o)
        if force or _newer(o, [src, *hdrs]):
            todo.append([HIPCC, *HIPFLAGS, "-c", str(src), "-o", str(o)])
    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, todo))
    so = LIB / "libpcmx_hip.so"
    cpu = LIB / "libpcmx_cpu.so"
    if force or todo or not so.exists() or _newer(so, [cpu]):
        _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", str(so), *map(str, objs),
              f"-L{tlib}", f"-L{LIB}", "-lamdhip64", "-lrccl", "-lpcmx_cpu",
              f"-Wl,-rpath,{tlib}", "-Wl,-rpath,$ORIGIN", "-Wl,--no-as-needed"])
    return so


FAULT_SRCS = ["kernels/scan.hip", "kernels/stencil.hip"]


def build_faultinj(force=False):
    """Test-only library: the same kernel sources compiled with -DPCMX_FAULT_INJECT (never loaded by the package)."""
    _, tlib, _ = _torch_paths()
    (OBJ / "fault").mkdir(parents=True, exist_ok=True)
    so = LIB / "libpcmx_faultinj.so"
    hdrs = _headers()
    objs = []
    todo = []
    for s in FAULT_SRCS:
        o = OBJ / "fault" / (s.replace("/", "_") + ".o")
        objs.append(o)
        if force or _newer(o, [CSRC / s, *hdrs]):
            todo.append([HIPCC, *HIPFLAGS, "-DPCMX_FAULT_INJECT", "-c", str(CSRC / s), "-o", str(o)])
    for cmd in todo:
        _run(cmd)
    if force or todo or not so.exists():
        _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", str(so), *map(str, objs), f"-L{tlib}", "-lamdhip64",
              f"-Wl,-rpath,{tlib}"])
    return so


def build_torch(force=False):
    incs, tlib, torch = _torch_paths()
    src = CSRC / "torch" / "ops.cpp"
    so = PKG / "_C.so"
    hip_so = LIB / "libpcmx_hip.so"
    if not (force or _newer(so, [src, hip_so, *_headers()])):
        return so
    pyinc = sysconfig.get_paths()["include"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [HIPCC, "-O2", "-fPIC", "-shared", "-std=c++17", "-x", "c++",
           *[f"-I{i}" for i in incs], f"-I{pyinc}", f"-I{CSRC / 'include'}", f"-I{ROCM / 'include'}",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H",
           str(src), "-o", str(so),
           f"-L{tlib}", f"-L{LIB}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
           "-ltorch_python", "-lamdhip64", "-lpcmx_hip", "-lpcmx_cpu",
           f"-Wl,-rpath,{tlib}", "-Wl,-rpath,$ORIGIN/lib"]
    _run(cmd)
    return so


BIN_TOOLS = {
    # name: (source, kind)  kind: c = host-only C tool, hip = links libpcmx_hip
    "spmv": ("bin/spmv_main.c", "c"),
    "histogram_serial": ("bin/histogram_main.c", "c"),
    "histogram_omp": ("bin/histogram_main.c", "c"),
    "histogram_pthreads": ("bin/histogram_main.c", "c"),
    "matrix_demo": ("bin/matrix_main.c", "c"),
    "vecops": ("bin/vecops_main.c", "c"),
    "raycast": ("bin/raycast_main.cpp", "hip"),
    "device_info": ("bin/device_info_main.cpp", "hip"),
    "region": ("bin/region_main.cpp", "hip"),
    "mpi_ring": ("bin/mpi_ring_main.cpp", "hip"),
    "collectives": ("bin/collectives_main.cpp", "hip"),
    "vmul": ("bin/vmul_main.cpp", "hip"),
    "pcmx_launch": ("bin/launch_main.c", "c"),
    # C programs written only against the reference 3-D entry points (pcmx_pipeline3d.h): host C, linked with
    # libpcmx_hip + libpcmx_cpu
    "pipeline3d": ("bin/pipeline3d_main.c", "c+hip"),
    "pipeline3d_opencl": ("bin/pipeline3d_main.c", "c+hip"),
    # vendor-library baseline (rocSPARSE generic SpMV): a standalone process on /opt/rocm's rocSPARSE + HIP runtime
    "spmv_vendor": ("bin/spmv_vendor_main.cpp", "rocm"),
}


def build_bin(force=False, jobs=8):
    BIN.mkdir(parents=True, exist_ok=True)
    _, tlib, _ = _torch_paths()
    todo = []
    for name, (src, kind) in BIN_TOOLS.items():
        s = CSRC / src
        if not s.exists():
            continue
        out = BIN / name
        deps = [s, LIB / "libpcmx_cpu.so", *_headers()] + ([LIB / "libpcmx_hip.so"] if "hip" in kind else [])
        if not (force or _newer(out, deps)):
            continue
        variant = f"-DPCMX_TOOL_{name.upper()}"
        rpath = "-Wl,-rpath,$ORIGIN/../parallel_c_programs_amd/lib"
        if kind == "c+hip":
            extra = ["-DPCMX_OPENCL_PROGRAM"] if name.endswith("_opencl") else []
            todo.append(["gcc", "-O2", "-std=gnu11", *extra, f"-I{CSRC / 'include'}", str(s), "-o", str(out),
                         f"-L{LIB}", f"-L{tlib}", "-lpcmx_hip", "-lpcmx_cpu", "-lamdhip64", "-lm", rpath,
                         f"-Wl,-rpath,{tlib}"])
        elif kind == "c":
            todo.append(["gcc", "-O2", "-std=gnu11", "-fopenmp", variant, f"-I{CSRC / 'include'}", str(s),
                         "-o", str(out), f"-L{LIB}", "-lpcmx_cpu", "-lm", rpath])
        elif kind == "rocm":
            todo.append([HIPCC, "-O2", "-std=c++17", "-Wno-deprecated-declarations", f"-I{CSRC / 'include'}", str(s),
                         "-o", str(out), f"-L{LIB}", f"-L{ROCM / 'lib'}", "-lrocsparse", "-lpcmx_cpu", rpath,
                         f"-Wl,-rpath,{ROCM / 'lib'}"])
        else:
            todo.append([HIPCC, "-O2", "-std=c++17", f"--offload-arch={ARCH}", variant, f"-I{CSRC / 'include'}",
                         str(s), "-o", str(out), f"-L{LIB}", f"-L{tlib}", "-lpcmx_hip", "-lpcmx_cpu", "-lamdhip64",
                         rpath, f"-Wl,-rpath,{tlib}"])
    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, todo))


def build_all(force=False, jobs=None, only=None):
    jobs = jobs or min(8, os.cpu_count() or 4)
    steps = only or ["cpu", "hip", "torch", "bin", "test"]
    if "cpu" in steps:
        build_cpu(force, jobs)
    if "hip" in steps:
        build_hip(force, jobs)
    if "torch" in steps:
        build_torch(force)
    if "bin" in steps:
        build_bin(force, jobs)
    if "test" in steps:
        build_faultinj(force)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--only", action="append", choices=["cpu", "hip", "torch", "bin", "test"])
    a = ap.parse_args(argv)
    build_all(a.force, a.jobs, a.only)
    print("pcmx build ok")


if __name__ == "__main__":
    sys.exit(main())
