"""Sanitizer builds of the host code: the C library + CPU tools rebuilt under
AddressSanitizer/UndefinedBehaviorSanitizer and ThreadSanitizer into build/san-<kind>/, then run on the
reference workloads. GPU code is not instrumented (GPU sanitizers are not available on the target pool);
the host side of the native comm layer (TCP transport, distributed region growing) is.

    python -m parallel_c_programs_amd.sanitize [asan|tsan]...
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

from ._build import CFLAGS, CPU_SRCS, CSRC, NO_CONTRACT, ROOT

SAN_FLAGS = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread", "-fno-omit-frame-pointer"],
}
TOOLS = {  # tool: (source, define)
    "matrix_demo": ("bin/matrix_main.c", "PCMX_TOOL_MATRIX_DEMO"),
    "spmv": ("bin/spmv_main.c", "PCMX_TOOL_SPMV"),
    "histogram_pthreads": ("bin/histogram_main.c", "PCMX_TOOL_HISTOGRAM_PTHREADS"),
    "histogram_omp": ("bin/histogram_main.c", "PCMX_TOOL_HISTOGRAM_OMP"),
    "pcmx_launch": ("bin/launch_main.c", "PCMX_TOOL_PCMX_LAUNCH"),
}


def _run(cmd, **kw):
    r = subprocess.run(cmd, capture_output=True, text=True, **kw)
    if r.returncode:
        raise RuntimeError(f"{' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def build(kind: str) -> Path:
    out = ROOT / "build" / f"san-{kind}"
    out.mkdir(parents=True, exist_ok=True)
    flags = [f for f in CFLAGS if f not in ("-O3",)] + ["-O1", "-g"] + SAN_FLAGS[kind]
    if kind == "tsan":  # libgomp is not TSan-instrumented: keep OpenMP out of the TSan build's own code
        flags = [f for f in flags if f != "-fopenmp"]
    objs = []
    for s in CPU_SRCS:
        o = out / (s.replace("/", "_") + ".o")
        extra = ["-ffp-contract=off"] if s in NO_CONTRACT else []
        _run(["gcc", *flags, *extra, "-c", str(CSRC / s), "-o", str(o)])
        objs.append(str(o))
    lib = out / "libpcmx_cpu.so"
    _run(["gcc", "-shared", *SAN_FLAGS[kind], *(["-fopenmp"] if kind == "asan" else []), "-o", str(lib), *objs,
          "-lm", "-lpthread"])
    # the distributed region binary is C++ + HIP for the device transports; the sanitizer build drives the
    # same host algorithm through a small C driver instead
    drv = out / "region_cpu.c"
    drv.write_text(REGION_DRIVER)
    tools = dict(TOOLS, region_cpu=(str(drv), "PCMX_TOOL_REGION_CPU"))
    for name, (src, define) in tools.items():
        srcp = src if os.path.isabs(src) else str(CSRC / src)
        _run(["gcc", *flags, f"-D{define}", srcp, "-o", str(out / name), f"-L{out}", "-lpcmx_cpu", "-lm",
              f"-Wl,-rpath,{out}"])
    return out


REGION_DRIVER = r"""
#include <stdio.h>
#include <stdlib.h>
#include "pcmx_comm.h"
#include "pcmx_cpu.h"
int main(int argc, char** argv) {
    pcmx_comm_t* c = NULL;
    if (argc < 2 || pcmx_comm_init_env_tcp(&c)) return 1;
    pcmx_region_backend_t be;
    pcmx_region_backend_host(&be);
    int W = 0, H = 0;
    unsigned char* img = c->rank == 0 ? pcmx_read_bmp_dims(argv[1], &W, &H) : NULL;
    unsigned char* reg = c->rank == 0 ? (unsigned char*)malloc((size_t)W * H) : NULL;
    int rc = pcmx_region2d_distributed(c, &be, img, H, W, 2, NULL, reg, NULL);
    if (!rc && c->rank == 0) {
        for (long i = 0; i < (long)W * H; ++i) img[i] *= (reg[i] == 0);
        write_bmp(img, W, H);
    }
    pcmx_free(img);
    free(reg);
    pcmx_comm_barrier(c);
    pcmx_comm_destroy(c);
    return rc ? 2 : 0;
}
"""


def run_checks(kind: str, workdir: Path) -> list[str]:
    """Runs the sanitized tools; returns a list of failures (empty = clean)."""
    out = build(kind)
    assets = ROOT / "assets"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1")
    runs = [
        [str(out / "matrix_demo")],
        [str(out / "spmv"), "2000", "41", "20", "10", "20", "10"],
        [str(out / "histogram_pthreads"), str(assets / "peppers.bmp"), "4"],
        [str(out / "pcmx_launch"), "-n", "4", str(out / "region_cpu"), str(assets / "pic1.bmp")],
    ]
    if kind == "asan":
        runs.append([str(out / "histogram_omp"), str(assets / "dark.bmp"), "4"])
    bad = []
    for cmd in runs:
        r = subprocess.run(cmd, capture_output=True, text=True, cwd=workdir, env=env, timeout=600)
        text = r.stdout + r.stderr
        if r.returncode != 0 or "ERROR: AddressSanitizer" in text or "runtime error:" in text or \
                "WARNING: ThreadSanitizer" in text:
            bad.append(f"{' '.join(cmd)} -> rc={r.returncode}\n{text[-3000:]}")
    return bad


def main(argv=None) -> int:
    kinds = (argv if argv is not None else sys.argv[1:]) or ["asan", "tsan"]
    import tempfile

    fails = []
    for k in kinds:
        with tempfile.TemporaryDirectory() as d:
            fails += run_checks(k, Path(d))
    for f in fails:
        print(f)
    print("sanitizers: clean" if not fails else f"sanitizers: {len(fails)} failure(s)")
    return 1 if fails else 0


if __name__ == "__main__":
    raise SystemExit(main())
