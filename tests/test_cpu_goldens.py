"""Golden tests of the host C library against the reference's own outputs.

The reference ships no test suite; these oracles were recovered from its programs and fixture files:
T1 region(pic1.bmp) == 2-mpi-region-growing/out.bmp (assets/region_pic1_golden.bmp), T2 3-D region box,
T3 histogram equalisation MD5s, T4 banded SpMV nnz, T5 serial ray-cast sums, T6 matrix demo stdout,
T7 vector-multiply demo.
"""
import hashlib

import numpy as np
import pytest
import torch
from conftest import run_cli

from parallel_c_programs_amd import ops
from parallel_c_programs_amd.utils import bmp


def md5(a):
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_bmp_roundtrip(tmp_path, assets):
    img = bmp.read(assets / "pic1.bmp")
    assert img.shape == (512, 512)
    bmp.write(tmp_path / "x.bmp", img)
    back = bmp.read(tmp_path / "x.bmp")
    assert np.array_equal(back, img)
    raw = (tmp_path / "x.bmp").read_bytes()
    assert raw[:2] == b"BM" and len(raw) == 1078 + 512 * 512 + 2
    assert int.from_bytes(raw[2:6], "little") == 512 * 512 + 56  # reference file_size formula
    assert int.from_bytes(raw[10:14], "little") == 1078
    assert raw[6:10] == b"\0\0\0\0"  # creator fields defined (B13)


def test_bmp_deterministic(tmp_path):
    img = (np.arange(64 * 32) % 256).astype(np.uint8).reshape(32, 64)
    bmp.write(tmp_path / "a.bmp", img)
    bmp.write(tmp_path / "b.bmp", img)
    assert (tmp_path / "a.bmp").read_bytes() == (tmp_path / "b.bmp").read_bytes()


def test_write_out_bmp_contract(tmp_path):
    bmp.write_out_bmp(np.zeros((8, 8), np.uint8))
    assert (tmp_path / "out.bmp").exists()


def test_t1_region_golden(assets):
    img = torch.from_numpy(bmp.read(assets / "pic1.bmp"))
    gold = bmp.read(assets / "region_pic1_golden.bmp")
    reg = ops.region2d(img)
    assert int(reg.sum()) == 64420
    assert np.array_equal(ops.apply_region_mask(img, reg).numpy(), gold)


@pytest.mark.parametrize("name,digest", [("dark", "d97277785d26b323358eb22d5de4adc0"),
                                         ("light", "d97277785d26b323358eb22d5de4adc0"),
                                         ("peppers", "016e872aac8ef0937d13adf00b74b901")])
@pytest.mark.parametrize("method,threads", [("serial", 1), ("omp", 1), ("omp", 4), ("omp", 8),
                                            ("pthreads", 1), ("pthreads", 3), ("pthreads", 8)])
def test_t3_histogram(assets, name, digest, method, threads):
    img = torch.from_numpy(bmp.read(assets / f"{name}.bmp"))
    out = ops.histeq(img, method, threads)
    assert md5(out.numpy()) == digest


def test_t3_histogram_value_255_no_overflow(assets):
    # pic2.bmp contains pixel value 255 (B14: the reference's 255-bin table overflows); 256 bins here
    img = torch.from_numpy(bmp.read(assets / "pic2.bmp"))
    assert int((img == 255).sum()) == 12774
    a = ops.histeq(img, "serial")
    assert torch.equal(a, ops.histeq(img, "omp", 4)) and torch.equal(a, ops.histeq(img, "pthreads", 5))


def test_t4_banded_spmv():
    m = ops.banded_csr(100000, 401, 200, 100, 200, 10)
    assert m.nnz == 61_955_590
    assert int((m.row_ptr[1:] - m.row_ptr[:-1]).max()) == 621
    x = ops.create_vector(100000)
    y_csr = ops.spmv(m, x)
    y_band = ops.spmv_banded(m.val, m.row_ptr, 100000, 401, 200, 100, 200, 10, x)
    assert (y_csr - y_band).abs().max().item() < 1e-3


@pytest.mark.parametrize("n,a,b,c,d,e", [(30, 3, 2, 2, 1, 1), (57, 7, 3, 4, 2, 3), (12, 41, 20, 10, 20, 5)])
def test_t4_small_band_structure(n, a, b, c, d, e):
    # independent model of the reference's limit bookkeeping (spmv.c:91-141): ten running limits,
    # left bands clipped at 0, right bands at n, all limits advanced by one per row
    m = ops.banded_csr(n, a, b, c, d, e)
    ah = a // 2
    lim = [0] * 10
    lim[5], lim[6], lim[7], lim[8], lim[9] = ah, ah + b, ah + b + c, ah + b + c + d, ah + b + c + d + e
    lim[0], lim[1], lim[2], lim[3], lim[4] = -lim[9], -lim[8], -lim[7], -lim[6], -lim[5]
    for k in range(5, 10):
        lim[k] += 1
    for i in range(n):
        cols = list(range(max(0, lim[0]), max(0, lim[1]))) + list(range(max(0, lim[2]), max(0, lim[3]))) + \
            list(range(max(0, lim[4]), min(lim[5], n))) + list(range(min(n, lim[6]), min(n, lim[7]))) + \
            list(range(min(n, lim[8]), min(n, lim[9])))
        got = m.col[m.row_ptr[i]:m.row_ptr[i + 1]].tolist()
        assert got == cols, i
        lim = [v + 1 for v in lim]


def test_t5_raycast_serial_reference_volume():
    vol = ops.create_volume(512, background="rand")
    reg, _ = ops.region3d(vol, threshold=1)
    assert int(reg.sum()) == 2_197_899  # T2
    img = ops.raycast(vol, reg, 64)
    assert int(img.sum()) == 127180 and int((img == 255).sum()) == 100


def test_t2_region_is_box():
    vol = ops.create_volume(512, background="hash")
    reg, _ = ops.region3d(vol, threshold=1)
    box = torch.zeros(512, 512, 512, dtype=torch.uint8)
    box[251:400, 251:400, 1:100] = 1
    assert torch.equal(reg, box)


def test_t6_matrix_demo_stdout():
    lines = run_cli("run_matrix", "--compat").stdout.splitlines()
    assert lines[0] == "Matrix m:"
    assert lines[1] == "0.000000\t1.000000\t2.000000\t3.000000\t"
    assert "Matrix m is sparse: 1" in lines and "Matrix o is sparse: 1" in lines
    assert "Error (m*o): -1" in lines
    i = lines.index("p rows: 3")
    assert lines[i + 1] == "14.000000\t74.000000\t134.000000\t194.000000\t"
    assert lines[i + 3] == "134.000000\t994.000000\t1854.000000\t2714.000000\t"
    assert lines[-1] == "0.000000\t0.000000\t0.000000\t0.000000\t0.000000\t"
    fixed = run_cli("run_matrix").stdout.splitlines()
    assert "Matrix m is sparse: 0" in fixed  # B1 fixed by default


def test_matrix_gemm_mode_host():
    """run_matrix --gemm: the matrix_t multiply at N^3 through the host backend, every element vs fp64."""
    import json

    r = json.loads(run_cli("run_matrix", "--gemm", 96, "--reps", 1, "--device", "cpu").stdout.splitlines()[-1])
    assert r["n"] == 96 and r["device"] == "cpu" and r["check_passed"] and r["max_rel_err_vs_fp64"] < 1e-5


def test_device_info_json_and_arch_gate_without_gpu():
    import json

    import torch

    if torch.cuda.is_available():
        pytest.skip("host-only expectations")
    r = json.loads(run_cli("run_device_info", "--json").stdout.splitlines()[-1])
    assert r == {"device_count": 0, "devices": [], "peer_access": []}
    assert run_cli("run_device_info", "--require-arch", "gfx950", check=False).returncode == 1
    assert run_cli("run_device_info", "--probe", check=False).returncode == 1


def test_t7_vmul_demo():
    i = torch.arange(1024, dtype=torch.float32)
    r = ops.vmul(i + 1, 1.0 / (i + 1))
    assert torch.allclose(r, torch.ones(1024), atol=1e-6)


def test_native_extension_loads_without_gpu():
    """_C.so and libpcmx_hip.so resolve every symbol (a launcher lost in an edit fails here, on CPU)."""
    import ctypes

    from parallel_c_programs_amd._native import LIB_DIR, ops

    ctypes.CDLL(str(LIB_DIR / "libpcmx_hip.so"), mode=ctypes.RTLD_GLOBAL)
    o = ops()
    for name in ("sgemm", "reduce", "scan_out", "stencil5_", "stencil5xT_", "spmv_csr", "region3d_grow_"):
        assert hasattr(o, name), name


def test_reference_host_entry_points_t2():
    """create_data / grow_region_serial with the reference signatures (libpcmx_cpu, pcmx_pipeline3d.h)."""
    import ctypes

    import numpy as np

    from parallel_c_programs_amd._native import cpu_lib

    lib = cpu_lib()
    lib.create_data.restype = ctypes.POINTER(ctypes.c_ubyte)
    lib.grow_region_serial.restype = ctypes.POINTER(ctypes.c_ubyte)
    lib.grow_region_serial.argtypes = [ctypes.POINTER(ctypes.c_ubyte)]
    data = lib.create_data()
    region = lib.grow_region_serial(data)
    n = 512 ** 3
    reg = np.ctypeslib.as_array(region, shape=(n,))
    assert int(np.count_nonzero(reg)) == 2197899
    vol = np.ctypeslib.as_array(data, shape=(n,)).reshape(512, 512, 512)
    assert int(vol[300, 300, 50]) == 35  # the seed voxel sits in the value-35 box (ref raycast.cu:140-143)
    lib.pcmx_free(ctypes.cast(data, ctypes.c_void_p))
    lib.pcmx_free(ctypes.cast(region, ctypes.c_void_p))


def test_sgemm_cli_host_backend():
    """run_sgemm without a GPU: the host C GEMM backend, reference Time line + JSON line with its fp64 error."""
    import json

    from conftest import run_cli

    out = run_cli("run_sgemm", 96, "--m", 40, "--steps", 1, "--warmup", 0, "--device", "cpu").stdout.splitlines()
    assert out[0].startswith("Time : ")
    line = json.loads(out[1])
    assert (line["m"], line["n"], line["k"], line["device"]) == (40, 96, 96, "cpu")
    assert line["max_rel_err_vs_fp64"] < 1e-5


@pytest.mark.parametrize("module,args,workloads", [
    ("run_stencil", (128, "--fuse", 2), ["stencil"]),
    ("run_reduce_scan", ("1e5", "--op", "both"), ["reduce", "scan"]),
    ("run_reduce_scan", ("1e5", "--op", "scan"), ["scan"]),
    ("run_spmv_dist", ("2e4", "2e5", "--chunks", 1), ["spmv"]),
])
def test_north_star_clis_on_host(module, args, workloads):
    """The north-star CLIs' own arguments map onto the workloads (reference Time line + one JSON line per workload,
    every numerics check passing) on the host path."""
    import json

    from conftest import run_cli

    out = run_cli(module, *args, "--steps", 1, "--warmup", 0, "--device", "cpu").stdout.splitlines()
    lines = [json.loads(s) for s in out if s.startswith("{")]
    assert [ln["workload"] for ln in lines] == workloads
    assert sum(s.startswith("Time : ") for s in out) == len(workloads)
    for ln in lines:
        errs = {k: v for k, v in ln.items() if "err" in k}
        assert all(v < 1e-5 for v in errs.values()), ln
        assert all(v for k, v in ln.items() if "bit_exact" in k), ln
