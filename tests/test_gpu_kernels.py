"""GPU numerics of the image/volume/stencil/sparse/halo kernels against the host C oracles and plain
PyTorch references (GPU only)."""
import pytest
import torch

from parallel_c_programs_amd import ops
from parallel_c_programs_amd.utils import bmp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["dark", "light", "peppers", "pic2"])
def test_histeq_bit_exact(gpu, assets, name):
    img = torch.from_numpy(bmp.read(assets / f"{name}.bmp").copy())
    ref = ops.histeq(img, "serial")
    for method in ("auto", "multiblock"):
        out = ops.histeq(img.to(gpu), method).cpu()
        assert torch.equal(out, ref), method


def test_histeq_large_random(gpu):
    g = torch.Generator().manual_seed(3)
    img = torch.randint(0, 256, (3000, 2999), dtype=torch.uint8, generator=g)
    ref = ops.histeq(img, "serial")
    assert torch.equal(ops.histeq(img.to(gpu)).cpu(), ref)
    assert torch.equal(ops.histeq(img.to(gpu), "multiblock").cpu(), ref)


@pytest.mark.parametrize("shape,hi", [((1, 7), 256), ((17, 3), 5), ((512, 512), 1), ((1023, 1021), 3),
                                      ((4096, 4096), 256)])
def test_histeq_tails_and_skew(gpu, shape, hi):
    """npix % 16 tails, one-block grids, single-bin images (every pixel on one per-lane counter) and repeated
    calls on the self-cleaning workspace, on the default and a side stream."""
    g = torch.Generator().manual_seed(shape[0] * 7 + hi)
    img = torch.randint(0, hi, shape, dtype=torch.uint8, generator=g) + (255 - hi if hi < 200 else 0)
    ref = ops.histeq(img, "serial")
    gi = img.to(gpu)
    for _ in range(3):
        assert torch.equal(ops.histeq(gi).cpu(), ref)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        out = ops.histeq(gi)
    s.synchronize()
    assert torch.equal(out.cpu(), ref)


def test_region2d_golden(gpu, assets):
    img = torch.from_numpy(bmp.read(assets / "pic1.bmp").copy())
    gold = torch.from_numpy(bmp.read(assets / "region_pic1_golden.bmp").copy())
    reg = ops.region2d(img.to(gpu)).cpu()
    assert int(reg.sum()) == 64420
    assert torch.equal(ops.apply_region_mask(img, reg), gold)


@pytest.mark.parametrize("name", ["pic2", "pic3", "pic4"])
def test_region2d_vs_serial(gpu, assets, name):
    img = torch.from_numpy(bmp.read(assets / f"{name}.bmp").copy())
    assert torch.equal(ops.region2d(img.to(gpu)).cpu(), ops.region2d(img))


def test_region2d_random_maze(gpu):
    g = torch.Generator().manual_seed(5)
    img = (torch.rand(700, 900, generator=g) < 0.45).to(torch.uint8) * 9  # 0/9 maze, threshold 2
    seeds = [(3, 3), (450, 350), (899, 699)]
    ref = ops.region2d(img, seeds=seeds)
    assert torch.equal(ops.region2d(img.to(gpu), seeds=seeds).cpu(), ref)


def test_volume_gen_matches_host(gpu):
    v_gpu = ops.create_volume(128, device=gpu, seed=7).cpu()
    v_cpu = ops.create_volume(128, device="cpu", seed=7)
    assert torch.equal(v_gpu, v_cpu)


@pytest.mark.parametrize("method", ["tiled", "naive"])
def test_region3d_small(gpu, method):
    vol = ops.create_volume(128, device="cpu", seed=3)
    ref, _ = ops.region3d(vol, seed=(50, 100, 100), threshold=1)
    reg, n = ops.region3d(vol.to(gpu), seed=(50, 100, 100), threshold=1, method=method)
    assert torch.equal((reg.cpu() != 0).to(torch.uint8), ref)
    assert n >= 1


@pytest.mark.parametrize("dim,thr,levels", [(96, 1, 2), (128, 1, 3), (64, 3, 8), (128, 2, 5)])
def test_region3d_tiled_random_maze(gpu, dim, thr, levels):
    # random low-entropy volumes (long snaking similar paths), partial x-tiles (96), seeds on tile faces /
    # volume edges (a seed on a face of a tile that cannot grow), several thresholds: the bit-parallel tiled
    # grow equals the serial flood fill
    g = torch.Generator().manual_seed(dim * 10 + thr)
    vol = (torch.randint(0, levels, (dim, dim, dim), generator=g) * 3).to(torch.uint8)
    for seed in [(0, 0, 0), (63, 8, 16), (dim - 1, dim - 1, dim - 1), (32, 7, 8), (min(64, dim - 1), 15, 7)]:
        ref, _ = ops.region3d(vol, seed=seed, threshold=thr)
        reg, n = ops.region3d(vol.to(gpu), seed=seed, threshold=thr, method="tiled")
        assert torch.equal((reg.cpu() != 0).to(torch.uint8), ref), seed


def test_region3d_reference_box(gpu):
    # T2: the region from seed (50,300,300) is exactly the 99x149x149 box (2,197,899 voxels)
    vol = ops.create_volume(512, device=gpu, seed=0)
    reg, launches = ops.region3d(vol, threshold=1, method="tiled")
    assert int((reg != 0).sum().item()) == 2_197_899
    box = torch.zeros(512, 512, 512, dtype=torch.bool, device=gpu)
    box[251:400, 251:400, 1:100] = True
    assert torch.equal(reg != 0, box)


@pytest.mark.parametrize("image_dim", [64, 128])
def test_raycast_global_bit_exact(gpu, image_dim):
    vol = ops.create_volume(512, device="cpu", seed=0)
    reg, _ = ops.region3d(vol, threshold=1)
    ref = ops.raycast(vol, reg, image_dim)
    out = ops.raycast(vol.to(gpu), reg.to(gpu), image_dim, method="global").cpu()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("image_dim", [64, 288])
def test_raycast_global_variants_bit_identical(gpu, image_dim):
    """Every global-caster variant (round 6: pair taps, one ray per 64 / 16 / 8 / 4-lane group, the DR16 interleaved
    volume) and the production rule give the one-step caster's image bit for bit, in both colour modes, on both sides
    of the 2^16-ray switch (288^2 = 82944 rays)."""
    vol = ops.create_volume(512, device=gpu, seed=0)
    reg, _ = ops.region3d(vol, threshold=1, method="tiled")
    reg = (reg != 0).to(torch.uint8)
    for method in ("global", "global_f32"):
        ref = ops.raycast(vol, reg, image_dim, method=method, variant=1)
        assert int(ref.long().sum()) > 0
        for v in [-1, 0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11]:
            out = ops.raycast(vol, reg, image_dim, method=method, variant=v)
            assert torch.equal(out, ref), (method, v)


def test_raycast_reference_data_golden(gpu):
    # T5: glibc-rand reference volume, 64x64 image sum = 127180 with 100 saturated pixels
    vol = ops.create_volume(512, background="rand")
    reg, _ = ops.region3d(vol.to(gpu), threshold=1)
    img = ops.raycast(vol.to(gpu), (reg != 0).to(torch.uint8), 64, method="global").cpu()
    assert int(img.sum()) == 127180 and int((img == 255).sum()) == 100


def test_raycast_texture_close(gpu):
    vol = ops.create_volume(512, device=gpu, seed=0)
    reg, _ = ops.region3d(vol, threshold=1)
    reg = (reg != 0).to(torch.uint8)
    a = ops.raycast(vol, reg, 128, method="global").float()
    b = ops.raycast(vol, reg, 128, method="texture").float()
    assert (a - b).abs().mean().item() < 6.0
    assert abs(a.mean().item() - b.mean().item()) < 3.0


@pytest.mark.parametrize("dim", [8, 16, 20, 21, 64, 72])
@pytest.mark.parametrize("hi", [128, 256])
def test_brick_pack_texels(gpu, dim, hi):
    # texel = 2x2x2 footprint of data then region, edge-clamped; narrow 8-B texels (region in bit 7) when every
    # data value < 128, else 16-B texels; 12-B-row (dim % 8 == 0, >= 16: narrow kernel + flag-gated wide kernel),
    # vector (dim % 4 == 0) and scalar pack kernels vs a plain torch gather
    g = torch.Generator().manual_seed(dim + hi)
    d = torch.randint(0, hi, (dim, dim, dim), dtype=torch.uint8, generator=g)
    r = (torch.rand(dim, dim, dim, generator=g) < 0.3).to(torch.uint8) * 7
    from parallel_c_programs_amd._native import ops as native

    tex = native().brick_pack(d.to(gpu), r.to(gpu)).cpu()
    n = dim ** 3
    assert tex.numel() == 2 * n + 2
    wide = int(tex[2 * n].item() & 0xFFFFFFFF)
    assert wide == (1 if hi > 128 else 0)
    i = torch.arange(dim)
    i1 = (i + 1).clamp(max=dim - 1)
    rb = (r != 0).to(torch.uint8)

    def corners(vol, zz):
        return torch.stack([vol[zz][:, yy][:, :, xx] for yy, xx in [(i, i), (i, i1), (i1, i), (i1, i1)]], -1)

    if wide:
        got = tex[:2 * n].view(torch.uint8).view(dim, dim, dim, 16)
        want = torch.cat([corners(d, i), corners(d, i1), corners(rb, i), corners(rb, i1)], -1)
    else:
        got = tex[:n].view(torch.uint8).view(dim, dim, dim, 8)
        want = torch.cat([corners(d, i) | (corners(rb, i) << 7), corners(d, i1) | (corners(rb, i1) << 7)], -1)
    assert torch.equal(got, want)


def test_raycast_texture_batches_identical(gpu):
    # the prefetch-batched march must give the image of the one-step-at-a-time march, bit for bit
    vol = ops.create_volume(512, device=gpu, seed=0)
    reg, _ = ops.region3d(vol, threshold=1)
    reg = (reg != 0).to(torch.uint8)
    imgs = [ops.raycast(vol, reg, 96, method="texture", batch=b) for b in (1, 4, 8, 16)]
    assert int(imgs[0].sum()) > 0
    for im in imgs[1:]:
        assert torch.equal(im, imgs[0])


def test_raycast_texture_segments_agree(gpu):
    # splitting every ray's steps over 1 / 2 / 4 waves composes the same colour up to f32 summation order
    vol = ops.create_volume(512, device=gpu, seed=0)
    reg, _ = ops.region3d(vol, threshold=1)
    reg = (reg != 0).to(torch.uint8)
    imgs = [ops.raycast(vol, reg, 128, method="texture", segments=s).int() for s in (1, 2, 4)]
    for im in imgs[1:]:
        d = (im - imgs[0]).abs()
        assert d.max().item() <= 1 and int((d > 0).sum()) <= 16
    wide = ops.raycast(vol | 128, reg, 64, method="texture", segments=4).int()  # 16-B texel path, same split
    wide1 = ops.raycast(vol | 128, reg, 64, method="texture", segments=1).int()
    assert (wide - wide1).abs().max().item() <= 1


@pytest.mark.parametrize("shape", [(256, 512), (1000, 1024), (515, 4096)])
def test_stencil_bit_exact(gpu, shape):
    rows, cols = shape
    u = ops.init_grid(rows, cols, device="cpu")
    ref = u.clone()
    for _ in range(3):
        ref = ops.stencil5_reference(ref, 0, rows)
    a = u.to(gpu)
    b = torch.empty_like(a)
    b.copy_(a)
    for _ in range(3):
        ops.stencil5_step_(a, b, 0, rows)
        a, b = b, a
    assert torch.equal(a.cpu()[1:-1], ref[1:-1])


def test_stencil_row_range_split(gpu):
    rows, cols = 512, 1024
    u = ops.init_grid(rows, cols, device=gpu)
    full = u.clone()
    ops.stencil5_step_(u, full, 0, rows)
    part = u.clone()
    ops.stencil5_step_(u, part, 0, rows, row_range=(1, rows - 1))
    ops.stencil5_step_(u, part, 0, rows, row_range=(0, 1))
    ops.stencil5_step_(u, part, 0, rows, row_range=(rows - 1, rows))
    assert torch.equal(full, part)


@pytest.mark.parametrize("steps", [2, 3, 4, 5, 6, 8])
@pytest.mark.parametrize("shape", [(256, 512), (1000, 1000), (515, 4096), (9, 2000), (4000, 800), (8300, 1000),
                                   (12400, 600)])
def test_stencil_fused_steps_bit_exact(gpu, shape, steps):
    """Temporal-blocking kernel == `steps` single steps (bf16 bits); random data so every lane/strip-overlap
    path counts; column counts that are not multiples of the 496 / 248 / 240-column output strips; the row counts
    cover every production launch shape (edge launches of <= 64 rows: 4 columns per lane, 2-row waves; under 3072
    rows 8 columns x 24 rows at T <= 4, 4 columns x 18 / 24 at T = 6 / 8; under 6144 and 12288 the 24 / 32-row
    shapes; 64 (T >= 6) / 24 above; interior waves: v2 fast path with the trapezoid skip, edge waves: v1 pipeline)."""
    rows, cols = shape
    g = torch.Generator().manual_seed(rows + steps)
    u = (torch.rand(rows + 2, cols, generator=g) * 4 - 2).to(torch.bfloat16)
    ref = u
    for _ in range(steps):
        ref = ops.stencil5_reference(ref, 0, rows)
    a = u.to(gpu)
    b = a.clone()
    ops.stencil5_fused_step_(a, b, 0, rows, halo=1, steps=steps)
    assert torch.equal(b.cpu()[1:-1].view(torch.int16), ref[1:-1].view(torch.int16))


@pytest.mark.parametrize("steps", [3, 4, 5, 6, 8])
@pytest.mark.parametrize("shape", [(515, 1000), (70, 2056), (200, 264)])
def test_stencil_fused_every_lane_geometry(gpu, shape, steps):
    """Every explicit launch shape (ops.stencil.launch_shape: 4 or 8 columns per lane x 2..133 rows per wave x prefetch
    ring 3 / 6 / 9, for full and edge launches; rows per wave is a launch parameter, so odd counts too) gives the bits of
    `steps` single steps: ragged column counts (stale-lane rule of 4-column lanes at T = 8: two stale lanes per strip
    side), Dirichlet rows and columns, strips ending inside a lane range. The shape is a per-launch argument: no state
    is left behind in the library."""
    from parallel_c_programs_amd.ops.stencil import launch_shape

    rows, cols = shape
    g = torch.Generator().manual_seed(rows + cols + steps)
    u = (torch.rand(rows + 2, cols, generator=g) * 4 - 2).to(torch.bfloat16)
    ref = u
    for _ in range(steps):
        ref = ops.stencil5_reference(ref, 0, rows)
    a = u.to(gpu)
    for cpl in (4, 8):
        for rpw in (2, 4, 7, 16, 18, 24, 32, 64, 67, 133):
            for ahead in ((0, 3, 9) if rpw in (7, 64) else (0,)):
                b = torch.zeros_like(a)
                ops.stencil5_fused_step_(a, b, 0, rows, halo=1, steps=steps, shape=launch_shape(cpl, rpw, ahead))
                assert torch.equal(b.cpu()[1:-1].view(torch.int16), ref[1:-1].view(torch.int16)), (cpl, rpw, ahead)
    b = torch.zeros_like(a)
    ops.stencil5_fused_step_(a, b, 0, rows, halo=1, steps=steps)  # the production rule after the sweep: same bits
    assert torch.equal(b.cpu()[1:-1].view(torch.int16), ref[1:-1].view(torch.int16))
    with pytest.raises(RuntimeError):
        ops.stencil5_fused_step_(a, b, 0, rows, halo=1, steps=steps, shape=5)  # 5 columns per lane: refused


@pytest.mark.parametrize("steps", [6])
def test_stencil_paired_waves_bit_identical(gpu, steps):
    """Paired waves (round 6, stencil5xT2p_kernel: two vertically adjacent waves march down / up and trade their
    common trapezoid through LDS; a measured, not adopted lab shape) give the bits of the unpaired kernel and of the CPU oracle: a rank's slab inside a
    larger grid (no Dirichlet row in reach, so the paired path runs), rows per wave from T up, last blocks whose lower
    wave has 1 row, several rows, or none, a two-span launch, and a slab touching the global edge (the unpaired
    fall-back of such blocks)."""
    from parallel_c_programs_amd.ops.stencil import launch_shape

    cols = 1032
    for rpw in sorted({steps, steps + 1, 18, 24, 64}):
        for rows in (4 * rpw + rpw + 1, 8 * rpw + 3, 4 * rpw + 2 * rpw, 2 * rpw):
            g = torch.Generator().manual_seed(rows * 31 + rpw + steps)
            u = (torch.rand(rows + 2 * steps, cols, generator=g) * 4 - 2).to(torch.bfloat16)
            for row0, grows in ((5000, 100000), (0, rows)):
                ref = u.clone()
                ops.stencil5_fused_step_(u, ref, row0, grows, halo=steps, steps=steps)  # CPU oracle
                a = u.to(gpu)
                for paired in (True, False):
                    b = torch.zeros_like(a)
                    ops.stencil5_fused_step_(a, b, row0, grows, halo=steps, steps=steps,
                                             shape=launch_shape(4, rpw, 0, paired))
                    got = b.cpu()[steps:-steps].view(torch.int16)
                    assert torch.equal(got, ref[steps:-steps].view(torch.int16)), (rpw, rows, row0, paired)
            # two spans in one launch (the distributed step's edge bands, here wide enough for pairs)
            row0, grows = 5000, 100000
            ref = u.clone()
            ops.stencil5_fused_step_(u, ref, row0, grows, halo=steps, steps=steps)
            a = u.to(gpu)
            b = a.clone()
            mid = rows // 2
            ops.stencil5_fused_spans_(a, b, ((0, mid - 7), (mid + 5, rows)), row0, grows, halo=steps, steps=steps,
                                      shape=launch_shape(4, rpw, 0, True))
            ops.stencil5_fused_step_(a, b, row0, grows, halo=steps, steps=steps, row_range=(mid - 7, mid + 5))
            assert torch.equal(b.cpu()[steps:-steps].view(torch.int16), ref[steps:-steps].view(torch.int16)), (rpw, rows)
    with pytest.raises(RuntimeError):  # paired waves exist for T = 6 with 4 columns per lane only (a lab shape)
        ops.stencil5_fused_step_(a, b, 5000, 100000, halo=steps, steps=steps, shape=launch_shape(8, 24, 0, True))


@pytest.mark.parametrize("steps", [2, 4, 6])
@pytest.mark.parametrize("global_row0,global_rows", [(0, 300), (40, 340), (40, 300)])
def test_stencil_fused_deep_halo_slab_and_row_split(gpu, global_row0, global_rows, steps):
    """A rank's slab with `steps` halo rows (neighbour rows present) and the interior/boundary split used for
    overlap gives the same bits as the CPU oracle."""
    rows, cols = 300 - global_row0 if global_rows == 300 else 300, 1024
    g = torch.Generator().manual_seed(global_row0 + global_rows)
    u = (torch.rand(rows + 2 * steps, cols, generator=g) * 4 - 2).to(torch.bfloat16)
    ref = u.clone()
    ops.stencil5_fused_step_(u, ref, global_row0, global_rows, halo=steps, steps=steps)  # CPU oracle
    a = u.to(gpu)
    full, part = a.clone(), a.clone()
    ops.stencil5_fused_step_(a, full, global_row0, global_rows, halo=steps, steps=steps)
    for rr in [(steps, rows - steps), (0, steps), (rows - steps, rows)]:
        ops.stencil5_fused_step_(a, part, global_row0, global_rows, halo=steps, steps=steps, row_range=rr)
    assert torch.equal(full, part)
    assert torch.equal(full.cpu()[steps:-steps].view(torch.int16), ref[steps:-steps].view(torch.int16))
    # both edge bands in ONE launch (two row spans), as the distributed step does after the halo arrives
    spans = a.clone()
    ops.stencil5_fused_step_(a, spans, global_row0, global_rows, halo=steps, steps=steps,
                             row_range=(steps, rows - steps))
    ops.stencil5_fused_spans_(a, spans, ((0, steps), (rows - steps, rows)), global_row0, global_rows, halo=steps,
                              steps=steps)
    assert torch.equal(full, spans)


@pytest.mark.parametrize("steps", [4, 6])
@pytest.mark.parametrize("spans", [((0, 700), (5000, 6500)), ((0, 0), (100, 7000)), ((6000, 7000), (0, 0)),
                                   ((0, 3), (7997, 8000))])
def test_stencil_fused_spans_match_full(gpu, steps, spans):
    """Row spans in one launch (short and >= 6144-row span totals, one empty span, spans ending at the slab
    edges) write exactly their rows, bit-identical to the full-range launch, and nothing else."""
    rows, cols = 8000, 1000
    g = torch.Generator().manual_seed(steps)
    u = (torch.rand(rows + 2 * steps, cols, generator=g) * 4 - 2).to(torch.bfloat16).to(gpu)
    full = u.clone()
    ops.stencil5_fused_step_(u, full, 100, 20000, halo=steps, steps=steps)
    sentinel = torch.full_like(u, 7.0)
    out = sentinel.clone()
    ops.stencil5_fused_spans_(u, out, spans, 100, 20000, halo=steps, steps=steps)
    mask = torch.zeros(rows + 2 * steps, dtype=torch.bool, device=gpu)
    for a0, a1 in spans:
        mask[steps + a0:steps + a1] = True
    assert torch.equal(out[mask], full[mask])
    assert torch.equal(out[~mask], sentinel[~mask])


@pytest.mark.parametrize("dims", [(20000, 41, 20, 10, 20, 5), (333, 41, 20, 10, 20, 5), (50, 9, 3, 5, 2, 3),
                                  (4000, 1301, 10, 200, 10, 50), (20000, 401, 200, 100, 200, 10),
                                  (3001, 301, 10, 50, 10, 3), (1500, 401, 200, 100, 200, 10)])
def test_spmv_banded_variants_vs_host(gpu, dims):
    """Every banded kernel variant (0: wave per row; 1/4-7: LDS-staged windows, 4-B loads, block rows x rows in
    flight; 8 / 9 / 10 / 11: block stream of 16 / 32 / 12 / 24 rows, 16-B loads over each row block's contiguous values) against the host product: interior
    rows, rows clipped at both matrix edges (n smaller than the band reach: variant 8 then runs the variant-1 body in
    every block), a row block past the last row, rows longer than 16 x 64 nonzeros (1301 + 400 + 100: the dispatcher
    falls back to the wave-per-row kernel), and rows shorter than 256 nonzeros (variant 8 falls back to 1)."""
    n = dims[0]
    m = ops.banded_csr(*dims)
    x = ops.create_vector(n)
    ref = ops.spmv(m, x)
    vals, ro, xg = m.val.to(gpu), m.row_ptr.to(gpu), x.to(gpu)
    for v in (0, 1, 4, 5, 6, 7, 8, 9, 10, 11):
        out = ops.spmv_banded(vals, ro, *dims, xg, variant=v).cpu()
        assert (out - ref).abs().max().item() < 1e-3 * max(1.0, ref.abs().max().item()), (v, dims)


def test_spmv_banded_stream_unaligned_values_fall_back(gpu):
    """Variant 8 on a value array that is not 16-B aligned (a view one float in): the variant-1 kernel runs, same
    result; nothing is read outside the array."""
    dims = (6000, 401, 200, 100, 200, 10)
    m = ops.banded_csr(*dims)
    x = ops.create_vector(dims[0])
    ref = ops.spmv(m, x)
    buf = torch.zeros(m.val.numel() + 1, device=gpu)
    buf[1:] = m.val.to(gpu)
    out = ops.spmv_banded(buf[1:], m.row_ptr.to(gpu), *dims, x.to(gpu), variant=8).cpu()
    assert (out - ref).abs().max().item() < 1e-3 * max(1.0, ref.abs().max().item())


def test_spmv_banded_stream_inside_graph_capture(gpu):
    """Variant 8's slot table is built on the first call per band geometry (a HIP allocation + an async copy): inside a
    stream capture of an UNCACHED geometry no allocation may run, so the launch takes variant 1 and the capture stays
    valid; the replayed graph gives the host product. The same geometry outside a capture then builds the table (on the
    stream) and variant 8 runs the stream kernel with the same result."""
    dims = (7001, 403, 200, 100, 200, 10)  # a geometry no other test uses (the table cache is per process)
    m = ops.banded_csr(*dims)
    x = ops.create_vector(dims[0])
    ref = ops.spmv(m, x)
    vals, ro, xg = m.val.to(gpu), m.row_ptr.to(gpu), x.to(gpu)
    side = torch.cuda.Stream(device=gpu)
    side.wait_stream(torch.cuda.current_stream(gpu))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            out = ops.spmv_banded(vals, ro, *dims, xg, variant=8)
    torch.cuda.current_stream(gpu).wait_stream(side)
    g.replay()
    torch.cuda.synchronize()
    tol = 1e-3 * max(1.0, ref.abs().max().item())
    assert (out.cpu() - ref).abs().max().item() < tol
    out2 = ops.spmv_banded(vals, ro, *dims, xg, variant=8).cpu()
    assert (out2 - ref).abs().max().item() < tol


def test_scan_check_per_stream(gpu):
    """scan(check=True) and scan_check wait on (and read the look-back error word of) the CURRENT stream only."""
    x = torch.rand(3 * 32768 + 11, device=gpu)
    y = ops.scan(x, check=True)
    side = torch.cuda.Stream(device=gpu)
    side.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(side):
        y2 = ops.scan(x)
        ops.scan_check(gpu)
    torch.cuda.current_stream(gpu).wait_stream(side)
    ops.scan_check(gpu)
    ref = torch.cumsum(x.double(), 0)
    assert torch.allclose(y.double(), ref, rtol=1e-5, atol=1e-3) and torch.equal(y, y2)


def test_spmv_banded_vs_host(gpu):
    m = ops.banded_csr(20000, 41, 20, 10, 20, 5)
    x = ops.create_vector(20000)
    ref = ops.spmv(m, x)
    out = ops.spmv_banded(m.val.to(gpu), m.row_ptr.to(gpu), 20000, 41, 20, 10, 20, 5, x.to(gpu)).cpu()
    assert (out - ref).abs().max().item() < 1e-3
    out_csr = ops.spmv(m.to(gpu), x.to(gpu)).cpu()
    assert (out_csr - ref).abs().max().item() < 1e-3


@pytest.mark.parametrize("slices,item", [(16, 512), (24, 1024), (16, 384), (16, 256)])
def test_spmv_fused_combine_bit_identical(gpu, slices, item):
    """The round-5 fused combine (combine + split-row fix-up + send-buffer pack in ONE launch) against the two-launch
    combine + fix-up and a gather of the same send lists: same y bits, same send-buffer bits, on a power-law matrix
    whose hub rows are split into many items (fix-up entries)."""
    from parallel_c_programs_amd.ops.sparse import SlicedCSR
    from parallel_c_programs_amd.ops.vector import gather_

    m = ops.powerlaw_csr(300_000, 4_000_000, alpha=2.1, seed=5)
    sc = SlicedCSR(m.to(gpu), slices, item_nnz=item)
    assert sc.fix.shape[0] > 0  # split rows present
    x = torch.rand(m.n_cols, device=gpu)
    sc.fused_combine = False
    ref = sc.spmv(x)
    sc.fused_combine = True
    got = sc.spmv(x)
    assert torch.equal(got, ref)
    # a send list: each row to 0..3 slots (random), as the distributed step's per-peer lists
    g = torch.Generator(device=gpu).manual_seed(1)
    reps = torch.randint(0, 4, (sc.n_rows,), device=gpu, generator=g)
    rows = torch.repeat_interleave(torch.arange(sc.n_rows, device=gpu), reps)
    slot_of = torch.randperm(rows.numel(), device=gpu, generator=g)  # entry k of the row-sorted list -> buffer slot
    ptr = torch.zeros(sc.n_rows + 1, dtype=torch.int64, device=gpu)
    ptr[1:] = reps.cumsum(0)
    buf = torch.full((rows.numel(),), float("nan"), device=gpu)
    y = torch.empty_like(ref)
    sc.spmv(x, y, send=(ptr.to(torch.int32), slot_of.to(torch.int32), buf))
    want = torch.empty_like(buf)
    idx = torch.empty_like(slot_of)
    idx[slot_of] = rows  # slot -> row
    gather_(ref, idx.to(torch.int32), want)
    assert torch.equal(y, ref) and torch.equal(buf, want)


def test_spmv_powerlaw_vs_dense(gpu):
    m = ops.powerlaw_csr(3000, 200_000, alpha=2.2, seed=11)
    x = torch.rand(3000)
    ref = m.dense().double() @ x.double()
    out = ops.spmv(m.to(gpu), x.to(gpu)).cpu().double()
    assert ((out - ref).abs() / (ref.abs() + 1)).max().item() < 1e-4


def test_spmv_long_rows(gpu):
    # rows longer than one work item (split + atomics) next to empty rows
    n = 50
    lens = torch.tensor([0, 5000, 3, 0, 2049, 1] + [7] * (n - 6))
    rp = torch.zeros(n + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(lens, 0)
    nnz = int(rp[-1])
    g = torch.Generator().manual_seed(2)
    col = torch.randint(0, 4000, (nnz,), dtype=torch.int32, generator=g)
    val = torch.rand(nnz, generator=g)
    m = ops.CSR(rp, col, val, 4000)
    x = torch.rand(4000, generator=g)
    ref = m.dense().double() @ x.double()
    out = ops.spmv(m.to(gpu), x.to(gpu)).cpu().double()
    assert (out - ref).abs().max().item() < 1e-3


@pytest.mark.parametrize("slices,head", [(8, 0.0), (16, 0.0625), (24, 0.0), (32, 0.2)])
def test_spmv_sliced_powerlaw_vs_fp64(gpu, slices, head):
    m = ops.powerlaw_csr(30000, 600_000, alpha=2.2, seed=5)
    x = torch.rand(30000, dtype=torch.float32)
    ref = ops.SlicedCSR(m, slices, head=head).reference(x)  # layout oracle (CPU)
    rows = torch.repeat_interleave(torch.arange(m.n_rows), m.row_ptr[1:] - m.row_ptr[:-1])
    want = torch.zeros(m.n_rows, dtype=torch.float64).index_add_(0, rows, m.val.double() * x.double()[m.col.long()])
    absrow = torch.zeros(m.n_rows, dtype=torch.float64).index_add_(0, rows, (m.val.double() * x.double()[m.col.long()]).abs())
    assert torch.allclose(ref, want, rtol=0, atol=1e-9)
    s = ops.SlicedCSR(m.to(gpu), slices, head=head)
    out = s.spmv(x.to(gpu)).cpu().double()
    assert torch.equal(out, s.spmv(x.to(gpu)).cpu().double())  # reproducible
    # fp32 accumulation: error bounded by a few ulps of the row's absolute sum
    assert ((out - want).abs() / (absrow + 1e-3)).max().item() < 1e-5
    plain = ops.spmv(m.to(gpu), x.to(gpu)).cpu().double()
    assert ((out - plain).abs() / (absrow + 1e-3)).max().item() < 1e-5
    # the packed index stream (production) and the unpacked col + lrow arrays: same products, same order
    assert s.cr is not None
    unpacked = ops.SlicedCSR(m.to(gpu), slices, head=head, pack=False)
    assert unpacked.cr is None
    assert torch.equal(out, unpacked.spmv(x.to(gpu)).cpu().double())
    # byte-packed-scan combine (production) vs the ballot-rank combine (mode bit 6): same partials, same order
    assert torch.equal(out, s.spmv(x.to(gpu), mode=64).cpu().double())
    assert torch.equal(out, unpacked.spmv(x.to(gpu), mode=64).cpu().double())
    # the short items of distributed ranks (384 / 256 nonzeros, 6 / 4 per lane; packed layout only): fp64 bound,
    # reproducible
    for item in (384, 256):
        si = ops.SlicedCSR(m.to(gpu), slices, head=head, item_nnz=item)
        oi = si.spmv(x.to(gpu)).cpu().double()
        assert torch.equal(oi, si.spmv(x.to(gpu)).cpu().double())
        assert ((oi - want).abs() / (absrow + 1e-3)).max().item() < 1e-5, item


@pytest.mark.parametrize("item_nnz", [512, 1024])
def test_spmv_sliced_packed_wide_slices(gpu, item_nnz):
    """Slices close to the 2^21-column limit of the packed word (few slices over 8e6 columns, head columns
    flagged) and 512-/1024-nnz items: packed == unpacked bit for bit, both close to fp64."""
    n_rows, n_cols = 2000, 8_000_000
    g = torch.Generator().manual_seed(11)
    lens = torch.randint(0, 400, (n_rows,), generator=g)
    rp = torch.zeros(n_rows + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(lens, 0)
    nnz = int(rp[-1])
    # half the nonzeros in a hot head (low columns), half uniform over all columns; sorted within each row
    col = torch.where(torch.rand(nnz, generator=g) < 0.5, torch.randint(0, 3000, (nnz,), generator=g),
                      torch.randint(0, n_cols, (nnz,), generator=g)).to(torch.int32)
    for r in range(0, n_rows, 1):
        a, b = int(rp[r]), int(rp[r + 1])
        col[a:b] = torch.sort(col[a:b]).values
    m = ops.CSR(rp, col, torch.rand(nnz, generator=g) - 0.5, n_cols)
    x = torch.rand(n_cols, generator=g)
    s = ops.SlicedCSR(m.to(gpu), 8, head=0.3, item_nnz=item_nnz)
    assert s.cr is not None and s.head_cols > 0
    u = ops.SlicedCSR(m.to(gpu), 8, head=0.3, item_nnz=item_nnz, pack=False)
    xg = x.to(gpu)
    out = s.spmv(xg).cpu().double()
    assert torch.equal(out, u.spmv(xg).cpu().double())
    rows = torch.repeat_interleave(torch.arange(n_rows), lens)
    want = torch.zeros(n_rows, dtype=torch.float64).index_add_(0, rows, m.val.double() * x.double()[m.col.long()])
    assert (out - want).abs().max().item() < 1e-3


def test_spmv_sliced_long_rows_and_unsorted_columns(gpu):
    # rows long enough to split into several items INSIDE one slice (fix-up path), empty rows, unsorted columns
    n = 64
    lens = torch.tensor([0, 40000, 3, 0, 17000, 1, 9000] + [5] * (n - 7))
    rp = torch.zeros(n + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(lens, 0)
    nnz = int(rp[-1])
    g = torch.Generator().manual_seed(7)
    col = torch.randint(0, 5000, (nnz,), dtype=torch.int32, generator=g)
    val = torch.rand(nnz, generator=g) - 0.5
    m = ops.CSR(rp, col, val, 5000)
    x = torch.rand(5000, generator=g)
    ref = m.dense().double() @ x.double()
    s = ops.SlicedCSR(m.to(gpu), 8, head=0.1)
    assert s.fix.shape[0] > 0
    outs = []
    for _ in range(3):  # partials / extras are reused scratch: a second call must not accumulate
        out = s.spmv(x.to(gpu)).cpu().double()
        assert (out - ref).abs().max().item() < 1e-3
        outs.append(out)
    # later pieces of split rows are summed per row in item order (no float atomics): bit-reproducible
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("dtype", [torch.uint8, torch.bfloat16, torch.float32])
def test_halo_pack_unpack(gpu, dtype):
    H, W = 37, 53
    t = (torch.arange((H + 2) * (W + 2)) % 251).to(dtype).view(H + 2, W + 2).contiguous()
    buf_ref = ops.pack_edges(t)
    buf = ops.pack_edges(t.to(gpu)).cpu()
    assert torch.equal(buf, buf_ref)
    dst = torch.zeros_like(t)
    ops.unpack_halo_(dst, buf_ref)
    dg = torch.zeros_like(t).to(gpu)
    ops.unpack_halo_(dg, buf_ref.to(gpu))
    assert torch.equal(dg.cpu(), dst)


@pytest.mark.parametrize("n", [1, 7, 4096, 1_000_003])
def test_gather_int32_vs_torch(gpu, n):
    """The SpMV send-buffer pack: out[i] = src[idx[i]] with int32 indices (ascending runs, repeats, the n % 4 tail),
    bit-equal to torch indexing; an index outside src reads 0."""
    g = torch.Generator(device=gpu).manual_seed(n)
    src = torch.rand(300_001, generator=g, device=gpu)
    idx = torch.sort(torch.randint(0, src.numel(), (n,), generator=g, device=gpu)).values.to(torch.int32)
    out = torch.empty(n, device=gpu)
    ops.gather_(src, idx, out)
    assert torch.equal(out, src[idx.long()])
    if n >= 4:
        bad = idx.clone()
        bad[n // 2] = src.numel() + 5
        ops.gather_(src, bad, out)
        assert out[n // 2].item() == 0.0 and torch.equal(out[:n // 2], src[idx[:n // 2].long()])
