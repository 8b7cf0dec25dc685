"""End-to-end GPU runs of the application layer: CLIs with the reference's argv/outputs and the north-star
workloads at reduced sizes, each with its numerics check (fp64 / host oracle)."""
import numpy as np
import pytest
import torch
from conftest import ASSETS, run_cli

from parallel_c_programs_amd import ops
from parallel_c_programs_amd.models import build_workload
from parallel_c_programs_amd.parallel import Context, grow_distributed
from parallel_c_programs_amd.utils import bmp
from parallel_c_programs_amd.utils.harness import timed

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return Context(device=torch.device("cuda", 0))


def test_region_cli_gpu_golden(gpu, tmp_path):
    run_cli("run_region", ASSETS / "pic1.bmp")
    assert np.array_equal(bmp.read(tmp_path / "out.bmp"), bmp.read(ASSETS / "region_pic1_golden.bmp"))


def test_grow_distributed_single_rank_gpu(gpu, ctx):
    img = torch.from_numpy(bmp.read(ASSETS / "pic2.bmp"))
    reg = grow_distributed(ctx, img, 2)
    assert torch.equal(reg.cpu(), ops.region2d(img))


@pytest.mark.parametrize("method", ["serial", "gpu"])
def test_histogram_cli(gpu, tmp_path, method):
    run_cli("run_histogram", ASSETS / "peppers.bmp", 4, "--method", method)
    out = bmp.read(tmp_path / "out.bmp")
    ref = ops.histeq(torch.from_numpy(bmp.read(ASSETS / "peppers.bmp")))
    assert np.array_equal(out, ref.numpy())


@pytest.mark.parametrize("precision", ["fp32", "bf16x6"])
def test_sgemm_cli(gpu, precision):
    """run_sgemm: the reference's Time line + one JSON line, odd shape padded by ops.sgemm, hipBLASLt comparison."""
    import json

    out = run_cli("run_sgemm", 1000, "--k", 700, "--precision", precision, "--steps", 2, "--warmup", 1,
                  "--compare").stdout.splitlines()
    assert out[0].startswith("Time : ") and out[0].endswith(" s")
    line = json.loads(out[1])
    assert line["precision"] == precision and line["kernel"] == f"variant {17 if precision == 'fp32' else 20}"
    assert line["max_rel_err_vs_fp64"] < 1e-5 and line["hipblaslt_max_rel_err_vs_fp64"] < 1e-5
    assert line["tflops"] > 0 and line["speedup_vs_hipblaslt"] > 0


def test_vmul_cli_table(gpu):
    lines = run_cli("run_vmul").stdout.splitlines()
    i = lines.index("Host\tDevice")
    assert lines[i + 1:i + 11] == ["1.00\t1.00"] * 10


def test_raycast_cli_opencl_variant(gpu, tmp_path):
    run_cli("run_raycast", "--opencl", timeout=900)
    img = bmp.read(tmp_path / "out.bmp")
    assert img.shape == (64, 64) and img.max() > 0


def test_raycast_cli_cuda_variant(gpu, tmp_path):
    r = run_cli("run_raycast", timeout=900)
    assert "Grow time:" in r.stdout and "Raycast time: " in r.stdout
    img = bmp.read(tmp_path / "out.bmp")
    assert img.shape == (512, 512) and img.max() > 0


def test_matrix_gemm_mode_gpu(gpu):
    """run_matrix --gemm on the GPU backend (the f32-MFMA kernel): every element vs fp64, rc 0."""
    import json

    r = run_cli("run_matrix", "--gemm", 1024, "--reps", 3)
    d = json.loads(r.stdout.splitlines()[-1])
    assert d["device"].startswith("cuda") and d["check_passed"] and d["tflops"] > 1.0


def test_device_info_json_arch_and_probe_gpu(gpu):
    import json

    d = json.loads(run_cli("run_device_info", "--json").stdout.splitlines()[-1])
    assert d["device_count"] >= 1 and d["devices"][0]["arch"].startswith("gfx950")
    assert d["peer_access"][0][0] is True
    assert run_cli("run_device_info", "--require-arch", "gfx950").returncode == 0
    assert run_cli("run_device_info", "--require-arch", "gfx942", check=False).returncode == 1
    p = [json.loads(ln) for ln in run_cli("run_device_info", "--probe").stdout.splitlines() if ln.startswith("{")]
    assert len(p) == d["device_count"]
    assert p[0]["hbm_read_gbps"] > 1000 and p[0]["hbm_write_gbps"] > 1000 and p[0]["sgemm_4096_tflops"] > 10


def test_spmv_cli_gpu(gpu):
    r = run_cli("run_spmv", 20000, 41, 20, 10, 20, 10, "--gpu")
    lines = r.stdout.splitlines()
    # host naive + host banded, then each GPU product in the reference's format ("Time : %f s" + compare())
    assert sum(ln.startswith("Time : ") for ln in lines) == 4
    assert any(ln.startswith("GPU CSR-adaptive") for ln in lines)
    assert any(ln.startswith("GPU banded, implicit columns") for ln in lines)
    assert sum(ln == "-10 more errors..." for ln in lines) == 3  # compare(): zero errors, all three products
    assert not any(ln.startswith("Error at:") for ln in lines)


@pytest.mark.parametrize("name,cfg,key,tol", [
    ("sgemm", {"n": 1024}, "max_rel_err_vs_fp64", 1e-5),
    ("reduce", {"n": 10_000_000}, "rel_err_vs_fp64", 1e-5),
    ("scan", {"n": 10_000_000}, "rel_err_vs_fp64", 1e-4),
])
def test_workloads_numerics(gpu, ctx, name, cfg, key, tol):
    w = build_workload(name, ctx, **cfg)
    secs = timed(ctx, w.step, 2, 1)
    rep = w.report(secs, 2)
    assert rep["value"] > 0
    assert w.check()[key] < tol


def test_stencil_workload_matches_reference(gpu, ctx):
    from parallel_c_programs_amd.parallel import reference_run

    w = build_workload("stencil", ctx, n=512)
    for _ in range(5):
        w.step()
    ref = reference_run(512, 5 * w.slab.fuse, device="cpu")
    assert torch.equal(w.slab.interior().cpu().view(torch.int16), ref.view(torch.int16))


def test_stencil_fused_graph_replay(gpu, ctx):
    from parallel_c_programs_amd.parallel import StencilSlab, reference_run

    s = StencilSlab(ctx, 256, 1024, fuse=2)
    s.run(10, graph=True)  # capture warm-up (4 updates) + 1 replay (4) + 1 eager fused step (2)
    assert s.steps_done == 10
    assert torch.equal(s.interior().cpu().view(torch.int16), reference_run(256, 10, 1024).view(torch.int16))


def test_stencil_hip_graph_replay_matches_eager(gpu, ctx):
    from parallel_c_programs_amd.parallel import StencilSlab, reference_run

    s = StencilSlab(ctx, 256, 512)
    s.run(7, graph=True)  # capture-warm-up pair + 2 replays + 1 eager step
    s.run(4, graph=True)  # the odd eager step swapped the buffers: re-capture, then replay
    assert s.steps_done == 11
    assert torch.equal(s.interior().cpu().view(torch.int16), reference_run(256, 11, 512).view(torch.int16))


def test_spmv_workload_matches_host(gpu, ctx):
    w = build_workload("spmv", ctx, n_rows=200_000, nnz=2_000_000)
    w.step()
    m = ops.powerlaw_csr(200_000, 2_000_000)
    x = w.d.from_padded(w.xp).cpu()  # one rank: the padded layout is the natural order
    ref = ops.spmv(m, x)
    assert torch.allclose(w.d.from_padded(w.y).cpu(), ref, rtol=1e-4, atol=1e-4)
    assert w.check()["max_rel_err_vs_fp64"] < 1e-5


def test_region3d_raycast_workloads(gpu, ctx):
    r = build_workload("region3d", ctx, dim=512)
    r.step()
    assert r.launches > 0 and int(r.region.sum()) > 0
    rc = build_workload("raycast", ctx, dim=512, image_dim=256)
    rc.step()
    assert rc.image.shape == (256, 256)


def test_matrix_multiply_dispatches_to_mfma_backend(gpu):
    """matrix_t's matrix_multiply (ref 1-introduction/matrix.c:63-81) hands large products to the MFMA SGEMM
    once libpcmx_hip registers itself as the GEMM backend; result checked against fp64."""
    import ctypes

    from parallel_c_programs_amd._native import cpu_lib, hip_lib

    class Mat(ctypes.Structure):
        _fields_ = [("data", ctypes.POINTER(ctypes.POINTER(ctypes.c_float))), ("rows", ctypes.c_int),
                    ("cols", ctypes.c_int)]

    lib, hip = cpu_lib(), hip_lib()
    lib.new_matrix.restype = ctypes.POINTER(Mat)
    lib.new_matrix.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.matrix_multiply.argtypes = [ctypes.POINTER(Mat), ctypes.POINTER(Mat), ctypes.POINTER(ctypes.POINTER(Mat))]
    lib.free_matrix.argtypes = [ctypes.POINTER(Mat)]
    hip.pcmx_register_gemm_backend.argtypes = [ctypes.c_longlong]
    hip.pcmx_register_gemm_backend(0)
    g = np.random.default_rng(3)
    a_np = g.standard_normal((300, 200), dtype=np.float32)
    b_np = g.standard_normal((200, 260), dtype=np.float32)
    a, b = lib.new_matrix(300, 200), lib.new_matrix(200, 260)
    ctypes.memmove(a.contents.data[0], a_np.ctypes.data, a_np.nbytes)
    ctypes.memmove(b.contents.data[0], b_np.ctypes.data, b_np.nbytes)
    ref = a_np.astype(np.float64) @ b_np.astype(np.float64)
    import os

    for prec in ("", "bf16x6"):  # the f32-MFMA kernel, then the fp32-accurate bf16 path (PCMX_SGEMM_PRECISION)
        os.environ["PCMX_SGEMM_PRECISION"] = prec
        try:
            c = ctypes.POINTER(Mat)()
            assert lib.matrix_multiply(a, b, ctypes.byref(c)) == 0
        finally:
            os.environ.pop("PCMX_SGEMM_PRECISION", None)
        out = np.ctypeslib.as_array(c.contents.data[0], shape=(300 * 260,)).reshape(300, 260).copy()
        assert np.abs(out - ref).max() / np.abs(ref).max() < 1e-5, prec
        lib.free_matrix(c)
    for m in (a, b):
        lib.free_matrix(m)


def _bin(name):
    from conftest import ROOT

    return str(ROOT / "bin" / name)


def test_native_vmul_table(gpu):
    import subprocess

    r = subprocess.run([_bin("vmul")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    i = lines.index("Host\tDevice")
    assert lines[i + 1:i + 11] == ["1.00\t1.00"] * 10
    assert any("gfx950" in ln for ln in lines[:i])


def test_native_raycast_opencl_variant_matches_ops(gpu, tmp_path):
    """bin/raycast --image-dim 64 --global --naive (the OpenCL program) == the torch-op pipeline, bit for bit."""
    import subprocess

    r = subprocess.run([_bin("raycast"), "--image-dim", "64", "--global", "--naive"], capture_output=True, text=True,
                       timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    img = bmp.read(tmp_path / "out.bmp")
    vol = ops.create_volume(512, device=gpu, seed=0)
    reg, _ = ops.region3d(vol, threshold=1, method="naive")
    want = ops.raycast(vol, (reg != 0).to(torch.uint8), 64, method="global").cpu().numpy()
    assert np.array_equal(img, want)


def test_native_raycast_cuda_program(gpu, tmp_path):
    import subprocess

    r = subprocess.run([_bin("raycast")], capture_output=True, text=True, timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert "Grow time:" in r.stdout and "Raycast time: " in r.stdout and r.stdout.count("Time : ") == 2
    img = bmp.read(tmp_path / "out.bmp")
    assert img.shape == (512, 512) and int((img == 255).sum()) > 0


def test_reference_entry_points_opencl_program(gpu, tmp_path):
    """bin/pipeline3d_opencl: a C program using only the reference names (IMAGE_DIM 64 via the header),
    grow_region_gpu + raycast_gpu: T2 region and the T5 64x64 image (sum 127,180, bit-identical to serial)."""
    import subprocess

    r = subprocess.run([_bin("pipeline3d_opencl")], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "region voxels: 2197899 (serial 2197899) identical" in r.stdout
    assert "serial caster sum: 127180, global caster bit-identical" in r.stdout
    assert bmp.read(tmp_path / "out.bmp").shape == (64, 64)


def test_reference_entry_points_cuda_program(gpu, tmp_path):
    """bin/pipeline3d: print_properties, create_data, grow_region_gpu_shared / grow_region_gpu (both equal to
    grow_region_serial), raycast_gpu_texture -> out.bmp, raycast_gpu = the serial 512^2 image (sum 8,154,839)."""
    import subprocess

    r = subprocess.run([_bin("pipeline3d")], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Device count:" in r.stdout and "Compute capability: 9.5" in r.stdout
    assert "Grow time:" in r.stdout and "Raycast time: " in r.stdout
    assert "region voxels: 2197899 (serial 2197899) identical" in r.stdout
    assert "(global-memory caster 8154839)" in r.stdout
    img = bmp.read(tmp_path / "out.bmp")
    assert img.shape == (512, 512) and int(img.astype(np.int64).sum()) > 0
