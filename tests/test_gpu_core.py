"""Numerics of the core gfx950 kernels against plain PyTorch fp32/fp64 references (GPU only)."""
import pytest
import torch

from parallel_c_programs_amd import ops
from parallel_c_programs_amd._native import ops as native_ops

pytestmark = pytest.mark.gpu


def test_extension_is_native(gpu):
    import parallel_c_programs_amd._C as C

    assert C.device_count() >= 1
    assert hasattr(native_ops(), "sgemm")


@pytest.mark.parametrize("n", [1, 3, 4, 1000, 4099, 1 << 20, (1 << 22) + 5])
def test_vmul_vadd_axpy(gpu, n):
    a = torch.rand(n, device=gpu)
    b = torch.rand(n, device=gpu)
    torch.testing.assert_close(ops.vmul(a, b), a * b)
    torch.testing.assert_close(ops.vadd(a, b), a + b)
    y = b.clone()
    ops.axpy_(y, 2.5, a)
    torch.testing.assert_close(y, 2.5 * a + b)


@pytest.mark.parametrize("n", [1, 5, 16384, 16387, 32768 * 3 + 4, (1 << 24) + 3, 256 * 32768 * 2 + 7])
def test_ticket_streams_copy_fill_exact(gpu, n):
    """The ticket-ordered streaming kernels (vector.hip): copy and fill bit-exact, vadd / vmul bit-exact against
    torch (one fp32 op per element), across single-tile, partial-tile, scalar-tail and more-tiles-than-CUs sizes;
    the self-resetting counter is exercised by back-to-back launches on one stream."""
    a = torch.rand(n, device=gpu)
    b = torch.rand(n, device=gpu)
    for _ in range(3):
        d = torch.full_like(a, float("nan"))
        ops.copy_(d, a)
        assert torch.equal(d, a)
        assert torch.equal(ops.vadd(a, b), a + b) and torch.equal(ops.vmul(a, b), a * b)
        ops.fill_(d, 1.25)
        assert bool((d == 1.25).all())


def test_copy_overlapping_ranges_is_memmove(gpu):
    """ops.copy_ between overlapping views of one buffer (tiles run in any order): the result is the source as it
    was before the copy, in both directions; an identical range is a no-op. Same for axpy_'s x overlapping y."""
    n = 3 * 32768 + 12
    base = torch.rand(n + 64, device=gpu)
    for shift in (4, -4, 32768):
        buf = base.clone()
        lo, hi = max(0, shift), max(0, -shift)
        src, dst = buf[hi:hi + n - abs(shift)], buf[lo:lo + n - abs(shift)]
        want = src.clone()
        ops.copy_(dst, src)
        assert torch.equal(dst, want), shift
    buf = base.clone()
    ops.copy_(buf, buf)
    assert torch.equal(buf, base)
    buf = base.clone()  # axpy_ with x a shifted view of y: x as it was before the update
    y, x = buf[0:n - 8], buf[8:n]
    want = y + 0.5 * x
    ops.axpy_(y, 0.5, x)
    torch.testing.assert_close(y, want, rtol=0, atol=0)


def test_ticket_streams_per_stream_counters_and_capture(gpu):
    """Launches on two streams at once (each stream has its own counter pair) and inside a hipGraph capture (the
    grid-stride form: no counter is allocated while capturing) all give exact results."""
    n = (1 << 23) + 1
    a, b = torch.rand(n, device=gpu), torch.rand(n, device=gpu)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    outs = []
    for s in (s1, s2, s1, s2):
        with torch.cuda.stream(s):
            outs.append(ops.vadd(a, b) if s is s1 else ops.vmul(a, b))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], a + b) and torch.equal(outs[2], a + b)
    assert torch.equal(outs[1], a * b) and torch.equal(outs[3], a * b)
    y = b.clone()
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        dst = torch.empty_like(a)
        with torch.cuda.graph(g, stream=cs):
            ops.copy_(dst, a)
            ops.axpy_(y, 2.0, a)
    y.copy_(b)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(dst, a)
    torch.testing.assert_close(y, 2.0 * a + b)


def test_vmul_reference_demo(gpu):
    # ref multiply_opencl.c:47-50: a[i] = i+1, b[i] = 1/(i+1) -> every product is 1.0
    i = torch.arange(1024, device=gpu, dtype=torch.float32)
    r = ops.vmul(i + 1, 1.0 / (i + 1))
    torch.testing.assert_close(r, torch.ones_like(r), atol=1e-6, rtol=0)


# first-pass partial counts 1, 1, 1, 31, 1221, 4096, 16384 (the cap): pass 2 folds float4s plus a 0-3 tail
@pytest.mark.parametrize("n", [1, 7, 4096, 123457, 5_000_011, 1 << 24, (1 << 26) + 3])
def test_reduce_sum_min_max(gpu, n):
    x = torch.randn(n, device=gpu)
    ref = x.double().sum().item()
    assert abs(ops.reduce(x, "sum").item() - ref) <= 1e-5 * max(1.0, x.abs().double().sum().item())
    assert ops.reduce(x, "min").item() == x.min().item()
    assert ops.reduce(x, "max").item() == x.max().item()
    xi = torch.randint(-1000, 1000, (n,), device=gpu, dtype=torch.int32)
    assert ops.reduce(xi, "sum").item() == xi.long().sum().item()
    assert ops.reduce(xi, "min").item() == xi.min().item()
    assert ops.reduce(xi, "max").item() == xi.max().item()


def test_reduce_deterministic(gpu):
    x = torch.randn(10_000_019, device=gpu)
    r = [ops.reduce(x, "sum").item() for _ in range(3)]
    assert r[0] == r[1] == r[2]


def test_dot(gpu):
    a = torch.randn(3_000_001, device=gpu)
    b = torch.randn(3_000_001, device=gpu)
    ref = (a.double() * b.double()).sum().item()
    assert abs(ops.dot(a, b).item() - ref) < 1e-3 * (a.abs() * b.abs()).double().sum().item() * 1e-2


@pytest.mark.parametrize("n", [1, 5, 8192, 8193, 100_003, 3 << 20])
@pytest.mark.parametrize("exclusive", [False, True])
def test_scan(gpu, n, exclusive):
    x = torch.rand(n, device=gpu) - 0.5
    ref = torch.cumsum(x.double(), 0)
    if exclusive:
        ref = torch.cat([ref.new_zeros(1), ref[:-1]])
    out = ops.scan(x, exclusive=exclusive)
    tol = 1e-5 * max(1.0, float(n) ** 0.5) * 4
    assert (out.double() - ref).abs().max().item() < tol


@pytest.mark.parametrize("exclusive", [False, True])
def test_scan_many_tiles_per_block(gpu, exclusive):
    # ~1221 128-KiB tiles over <= 256 persistent blocks: every block walks several tickets (taken two tiles
    # ahead), and the last tile is partial with a straddling f32x4 row
    n = 40_000_007
    x = torch.randint(0, 4, (n,), device=gpu).float()
    ref = torch.cumsum(x.long(), 0)
    if exclusive:
        ref = torch.cat([ref.new_zeros(1), ref[:-1]])
    out = ops.scan(x, exclusive=exclusive)
    # integer inputs: exact while partial sums stay below 2^24, then f32 rounding of the carried prefix
    err = (out.double() - ref.double()).abs() / ref.double().clamp_min(1.0)
    assert err.max().item() < 2e-5  # <= ~1 rounding of the carried prefix per tile hop
    assert torch.equal(out[: 1 << 20].long(), ref[: 1 << 20])


def test_scan_with_device_init(gpu):
    x = torch.ones(50_000, device=gpu)
    init = torch.tensor([10.0], device=gpu)
    out = ops.scan(x, init=init)
    assert out[0].item() == 11.0 and out[-1].item() == 50_010.0


def test_scan_integer_exact(gpu):
    # small integers sum exactly in f32 -> bit-exact against the integer cumsum
    x = torch.randint(0, 3, (2_000_000,), device=gpu).float()
    out = ops.scan(x)
    assert torch.equal(out.long(), torch.cumsum(x.long(), 0))


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 8])
def test_scan_schedules_exact(gpu, variant):
    """Every scan schedule (persistent / parked-tile / parked + early polls) on ragged sizes, exclusive, a device
    init and in place; small integers keep every prefix exact in f32."""
    import ctypes

    from parallel_c_programs_amd._native import hip_lib

    lib = hip_lib()
    lib.pcmx_scan_workspace_bytes.restype = ctypes.c_longlong
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for m in (1, 5, 32768, 32769, 300_001, 32768 * 700 + 13):
        x = torch.randint(-8, 9, (m,), device=gpu).float()
        ws = torch.empty(lib.pcmx_scan_workspace_bytes(ctypes.c_longlong(m)), dtype=torch.uint8, device=gpu)
        init = torch.tensor([3.0], device=gpu)
        ref = torch.cumsum(x.double(), 0)
        for exclusive, y, src, want in ((0, torch.empty_like(x), x, ref + 3.0),
                                        (1, torch.empty_like(x), x, torch.cat([ref.new_zeros(1), ref[:-1]]) + 3.0),
                                        (0, None, x.clone(), ref + 3.0)):
            y = src if y is None else y  # in place
            rc = lib.pcmx_scan_f32_variant(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                           ctypes.c_longlong(m), exclusive, ctypes.c_void_p(init.data_ptr()),
                                           ctypes.c_void_p(ws.data_ptr()), None, variant, stream)
            assert rc == 0
            assert lib.pcmx_scan_check(ctypes.c_void_p(ws.data_ptr()), stream) == 0
            assert torch.equal(y.double(), want), (m, exclusive)


@pytest.mark.parametrize("variant", [0, 1, 16, 17, 18])
def test_sgemm_identity_asymmetric(gpu, variant):
    # A = I with an asymmetric B catches a transposed C write (cdna_hip_programming.md §3)
    n = 256
    a = torch.eye(n, device=gpu)
    b = torch.arange(n * n, device=gpu, dtype=torch.float32).view(n, n) / 7.0
    c = ops.sgemm(a, b, variant=variant)
    assert torch.equal(c, b)
    c2 = ops.sgemm(b, a, variant=variant)
    assert torch.equal(c2, b)


@pytest.mark.parametrize("variant", [0, 16, 17, 18, 20])
def test_sgemm_register_staged_multitile_vs_fp64(gpu, variant):
    # several tiles in both directions and 2+ LDS stages of prefetch: M != N != K
    g = torch.Generator(device=gpu).manual_seed(variant)
    a = torch.rand(768, 1280, device=gpu, generator=g) * 2 - 1
    b = torch.rand(1280, 512, device=gpu, generator=g) * 2 - 1
    c = ops.sgemm(a, b, variant=variant)
    ref = a.double() @ b.double()
    assert ((c.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5


@pytest.mark.parametrize("shape", [(256, 256, 256), (512, 768, 1024), (1024, 1024, 2048), (100, 70, 33), (1000, 1000, 1000),
                                   (3500, 3600, 1000)])  # last: padded to 256-tiles + K % 64 -> direct-register kernel
def test_sgemm_vs_fp64(gpu, shape):
    m, n, k = shape
    a = torch.rand(m, k, device=gpu) * 2 - 1
    b = torch.rand(k, n, device=gpu) * 2 - 1
    c = ops.sgemm(a, b)
    ref = a.double() @ b.double()
    scale = (a.abs().double() @ b.abs().double())
    err = ((c.double() - ref).abs() / scale.clamp_min(1e-30)).max().item()
    assert err < 4e-6 * max(1.0, (k / 256) ** 0.5)


@pytest.mark.parametrize("shape", [(768, 1280, 512), (4352, 4096, 128)])
def test_sgemm_direct_persistent_many_tiles(gpu, shape):
    """Variant 18 caps the persistent direct kernel at 7 blocks (2-3 tiles per block at 768x1280; the cross-tile
    look-ahead and the past-the-end clamp); 4352x4096 runs 272 tiles on the production grid (one block per CU, some
    blocks two tiles). alpha/beta through the same epilogue."""
    m, n, k = shape
    g = torch.Generator(device=gpu).manual_seed(m + n)
    a = torch.rand(m, k, device=gpu, generator=g) * 2 - 1
    b = torch.rand(k, n, device=gpu, generator=g) * 2 - 1
    c0 = torch.rand(m, n, device=gpu, generator=g)
    ref = 1.5 * (a.double() @ b.double()) - 0.25 * c0.double()
    for variant in (17, 18):
        out = ops.sgemm_out(a, b, c0.clone(), alpha=1.5, beta=-0.25, variant=variant)
        err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-5, (variant, err)
        plain = ops.sgemm(a, b, variant=variant)
        assert torch.equal(plain, ops.sgemm(a, b, variant=17 if variant == 18 else 18))  # same sums, any grid


@pytest.mark.parametrize("shape", [(256, 256, 32), (512, 768, 96), (1024, 512, 2048), (300, 200, 70)])
def test_sgemm_x6_elementwise_fp32_accuracy(gpu, shape):
    """Variant 20 (fp32 GEMM on the bf16 matrix cores, exact 3-way operand split, 6 piece products): per-element
    error against the fp64 product, in units of sum |a||b|, within the native f32 MFMA kernel's bound."""
    m, n, k = shape
    g = torch.Generator(device=gpu).manual_seed(k)
    a = torch.rand(m, k, device=gpu, generator=g) * 2 - 1
    b = torch.rand(k, n, device=gpu, generator=g) * 2 - 1
    c = ops.sgemm(a, b, variant=20)
    ref = a.double() @ b.double()
    scale = a.abs().double() @ b.abs().double()
    err = ((c.double() - ref).abs() / scale.clamp_min(1e-30)).max().item()
    assert err < 4e-6 * max(1.0, (k / 256) ** 0.5), err


def test_sgemm_x6_alpha_beta(gpu):
    """Variant 20 through the alpha/beta epilogue (C read back, scaled, added) on a 4x2-tile problem."""
    g = torch.Generator(device=gpu).manual_seed(20)
    a = torch.rand(1024, 320, device=gpu, generator=g) * 2 - 1
    b = torch.rand(320, 512, device=gpu, generator=g) * 2 - 1
    c0 = torch.rand(1024, 512, device=gpu, generator=g)
    ref = 1.5 * (a.double() @ b.double()) - 0.25 * c0.double()
    out = ops.sgemm_out(a, b, c0.clone(), alpha=1.5, beta=-0.25, variant=20)
    assert ((out.double() - ref).abs().max() / ref.abs().max()).item() < 1e-6


def test_sgemm_x6_split_exact_wide_range(gpu):
    """The split is exact for |x| >= 2^-110: a diagonal A spanning 2^-40 .. 2^40 times B with columns spanning the
    same range multiplies within a few fp32 roundings of the fp64 product (6 piece products summed in f32: <= ~4
    ulp; measured 2.2), and power-of-two scales reproduce the exact products bit for bit (identity A included)."""
    n = 256
    scales = torch.pow(2.0, torch.linspace(-40, 40, n, device=gpu)).float()
    b = (torch.rand(n, n, device=gpu) * 2 - 1) * scales[None, :]
    a = torch.eye(n, device=gpu) * scales[:, None]
    c = ops.sgemm(a, b, variant=20)
    ref = a.double() @ b.double()
    assert ((c.double() - ref).abs() / ref.abs().clamp_min(1e-300)).max().item() < 2.5e-7
    # exact powers of two (torch.pow(2., x) on the GPU is an exp2 approximation: 2^29 -> 536870880)
    p2 = torch.tensor([2.0 ** e for e in torch.randint(-40, 41, (n,)).tolist()], device=gpu)
    exact = torch.eye(n, device=gpu) * p2[:, None]
    assert torch.equal(ops.sgemm(exact, b, variant=20), p2[:, None] * b)
    assert torch.equal(ops.sgemm(torch.eye(n, device=gpu), b, variant=20), b)


def test_sgemm_beta(gpu):
    a = torch.rand(256, 256, device=gpu)
    b = torch.rand(256, 256, device=gpu)
    c = torch.rand(256, 256, device=gpu)
    ref = 2.0 * (a.double() @ b.double()) + 0.5 * c.double()
    out = ops.sgemm_out(a, b, c.clone(), alpha=2.0, beta=0.5)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-4)


def test_sgemm_simt_baseline(gpu):
    a = torch.rand(300, 200, device=gpu)
    b = torch.rand(200, 100, device=gpu)
    torch.testing.assert_close(ops.sgemm_simt(a, b), a @ b, rtol=1e-4, atol=1e-4)
