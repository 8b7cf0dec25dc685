// Torch op registrations: every MI355X kernel of libpcmx_hip.so is exposed as torch.ops.pcmx.<name>.
// GPU tensors dispatch here (DispatchKey "CUDA" is the HIP device on ROCm builds of PyTorch); kernels
// run on the current torch HIP stream so they compose with torch.distributed (RCCL) streams and hipGraph
// capture. Workspaces come from the torch caching allocator (no hipMalloc on the launch path).
#include <cmath>
#include <map>
#include <mutex>
#include <torch/extension.h>
#include <torch/library.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "pcmx_hip.h"

namespace {

hipStream_t cur_stream(const at::Tensor& t) {
    return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_rc(int rc, const char* what) {
    TORCH_CHECK(rc == 0, "pcmx::", what, " failed: ", pcmx_error_string(rc), " (", rc, ")");
}

void check_gpu(const at::Tensor& t, const char* name, at::ScalarType dt) {
    TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
    TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}

at::Tensor aligned_contig(const at::Tensor& t) {
    at::Tensor c = t.contiguous();
    if (reinterpret_cast<uintptr_t>(c.data_ptr()) & 15u) c = c.clone();
    return c;
}

at::Tensor workspace(const at::Tensor& like, long long bytes) {
    return at::empty({std::max<long long>(bytes, 16)}, like.options().dtype(at::kByte));
}

// ---------------------------------------------------------------- element-wise
at::Tensor vmul(const at::Tensor& a, const at::Tensor& b) {
    check_gpu(a, "a", at::kFloat), check_gpu(b, "b", at::kFloat);
    TORCH_CHECK(a.numel() == b.numel(), "vmul: size mismatch");
    const at::DeviceGuard g(a.device());
    auto ac = aligned_contig(a), bc = aligned_contig(b);
    auto r = at::empty_like(ac);
    check_rc(pcmx_vmul_f32(ac.data_ptr<float>(), bc.data_ptr<float>(), r.data_ptr<float>(), ac.numel(), cur_stream(a)), "vmul");
    return r;
}

at::Tensor vadd(const at::Tensor& a, const at::Tensor& b) {
    check_gpu(a, "a", at::kFloat), check_gpu(b, "b", at::kFloat);
    TORCH_CHECK(a.numel() == b.numel(), "vadd: size mismatch");
    const at::DeviceGuard g(a.device());
    auto ac = aligned_contig(a), bc = aligned_contig(b);
    auto r = at::empty_like(ac);
    check_rc(pcmx_vadd_f32(ac.data_ptr<float>(), bc.data_ptr<float>(), r.data_ptr<float>(), ac.numel(), cur_stream(a)), "vadd");
    return r;
}

at::Tensor gather_(const at::Tensor& src, const at::Tensor& idx, at::Tensor out) {
    check_gpu(src, "src", at::kFloat), check_gpu(idx, "idx", at::kInt), check_gpu(out, "out", at::kFloat);
    TORCH_CHECK(src.is_contiguous() && idx.is_contiguous() && out.is_contiguous() && idx.numel() == out.numel(),
                "gather_: contiguous src / idx / out, out.numel() == idx.numel()");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(idx.data_ptr()) & 15u) == 0 && (reinterpret_cast<uintptr_t>(out.data_ptr()) & 15u) == 0,
                "gather_: idx and out must be 16-B aligned");
    const at::DeviceGuard g(src.device());
    check_rc(pcmx_gather_f32(src.data_ptr<float>(), src.numel(), idx.data_ptr<int>(), out.data_ptr<float>(), out.numel(),
                             cur_stream(src)),
             "gather_");
    return out;
}

// The streaming kernels take their tiles in any order: an input that PARTLY overlaps the output is copied out first
// (an input identical to the output, element for element, is fine: each element is read before it is written).
at::Tensor unaliased(const at::Tensor& in, const at::Tensor& out) {
    const auto i0 = reinterpret_cast<uintptr_t>(in.data_ptr()), o0 = reinterpret_cast<uintptr_t>(out.data_ptr());
    const uintptr_t ib = (uintptr_t)in.numel() * in.element_size(), ob = (uintptr_t)out.numel() * out.element_size();
    return (i0 != o0 && i0 < o0 + ob && o0 < i0 + ib) ? in.clone() : in;
}

at::Tensor axpy_(at::Tensor y, double alpha, const at::Tensor& x) {
    check_gpu(y, "y", at::kFloat), check_gpu(x, "x", at::kFloat);
    TORCH_CHECK(y.is_contiguous() && (reinterpret_cast<uintptr_t>(y.data_ptr()) & 15u) == 0, "axpy_: y must be contiguous, 16-B aligned");
    TORCH_CHECK(x.numel() == y.numel(), "axpy_: size mismatch");
    const at::DeviceGuard g(y.device());
    auto xc = unaliased(aligned_contig(x), y);
    check_rc(pcmx_axpy_f32((float)alpha, xc.data_ptr<float>(), y.data_ptr<float>(), y.numel(), cur_stream(y)), "axpy_");
    return y;
}

at::Tensor copy_(at::Tensor dst, const at::Tensor& src) {
    check_gpu(dst, "dst", at::kFloat), check_gpu(src, "src", at::kFloat);
    TORCH_CHECK(dst.is_contiguous() && (reinterpret_cast<uintptr_t>(dst.data_ptr()) & 15u) == 0, "copy_: dst must be contiguous, 16-B aligned");
    TORCH_CHECK(src.numel() == dst.numel() && src.device() == dst.device(), "copy_: size / device mismatch");
    const at::DeviceGuard g(dst.device());
    auto sc = unaliased(aligned_contig(src), dst);  // memmove semantics
    check_rc(pcmx_copy_f32(sc.data_ptr<float>(), dst.data_ptr<float>(), dst.numel(), cur_stream(dst)), "copy_");
    return dst;
}

at::Tensor fill_(at::Tensor x, double v) {
    check_gpu(x, "x", at::kFloat);
    TORCH_CHECK(x.is_contiguous() && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15u) == 0, "fill_: contiguous, aligned");
    const at::DeviceGuard g(x.device());
    check_rc(pcmx_fill_f32(x.data_ptr<float>(), (float)v, x.numel(), cur_stream(x)), "fill_");
    return x;
}

at::Tensor rand_uniform_(at::Tensor x, int64_t seed, double lo, double hi) {
    check_gpu(x, "x", at::kFloat);
    TORCH_CHECK(x.is_contiguous(), "rand_uniform_: contiguous");
    const at::DeviceGuard g(x.device());
    check_rc(pcmx_rand_uniform_f32(x.data_ptr<float>(), x.numel(), (unsigned long long)seed, (float)lo, (float)hi, cur_stream(x)),
             "rand_uniform_");
    return x;
}

// ---------------------------------------------------------------- reductions / scan
at::Tensor reduce(const at::Tensor& x, int64_t op) {
    TORCH_CHECK(x.is_cuda(), "reduce: GPU tensor expected");
    const at::DeviceGuard g(x.device());
    auto xc = aligned_contig(x);
    auto ws = workspace(x, pcmx_reduce_workspace_bytes(xc.numel()));
    if (x.scalar_type() == at::kFloat) {
        auto out = at::empty({}, x.options());
        check_rc(pcmx_reduce_f32(xc.data_ptr<float>(), xc.numel(), (int)op, out.data_ptr<float>(), ws.data_ptr(), cur_stream(x)), "reduce");
        return out;
    }
    TORCH_CHECK(x.scalar_type() == at::kInt, "reduce: float32 or int32 expected");
    auto out = at::empty({}, x.options());
    check_rc(pcmx_reduce_i32(xc.data_ptr<int32_t>(), xc.numel(), (int)op, out.data_ptr<int32_t>(), ws.data_ptr(), cur_stream(x)), "reduce");
    return out;
}

at::Tensor dot(const at::Tensor& a, const at::Tensor& b) {
    check_gpu(a, "a", at::kFloat), check_gpu(b, "b", at::kFloat);
    TORCH_CHECK(a.numel() == b.numel(), "dot: size mismatch");
    const at::DeviceGuard g(a.device());
    auto ac = aligned_contig(a), bc = aligned_contig(b);
    auto ws = workspace(a, pcmx_reduce_workspace_bytes(ac.numel()));
    auto out = at::empty({}, a.options());
    check_rc(pcmx_dot_f32(ac.data_ptr<float>(), bc.data_ptr<float>(), ac.numel(), out.data_ptr<float>(), ws.data_ptr(), cur_stream(a)), "dot");
    return out;
}

// Sticky look-back-timeout word per (device, stream) in host-mapped pinned memory: a scan kernel whose look-back
// gives up ORs 1 into it (system-scope atomic), so the host sees it without a copy. scan_check (and
// ops.scan(check=True)) synchronises THAT stream and raises; the next scan on the same stream raises too. One word
// per stream, so a failed scan on one stream is never reported (and cleared) by an unrelated call on another.
struct ScanErrWord {
    unsigned* host = nullptr;
    unsigned* dev = nullptr;
};

ScanErrWord& scan_err_word(int dev, hipStream_t stream) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, ScanErrWord> words;
    TORCH_CHECK(dev >= 0, "scan: device index");
    std::lock_guard<std::mutex> lock(mu);
    ScanErrWord& w = words[{dev, stream}];
    if (!w.host) {
        void* p = nullptr;
        TORCH_CHECK(hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess,
                    "scan: pinned error word");
        *static_cast<volatile unsigned*>(p) = 0u;
        void* d = nullptr;
        TORCH_CHECK(hipHostGetDevicePointer(&d, p, 0) == hipSuccess, "scan: mapped error word");
        w.host = static_cast<unsigned*>(p), w.dev = static_cast<unsigned*>(d);
    }
    return w;
}

void raise_pending_scan_error(int dev, hipStream_t stream) {
    volatile unsigned* w = scan_err_word(dev, stream).host;
    if (*w) {
        *w = 0u;
        TORCH_CHECK(false, "pcmx::scan: a scan on device ", dev, " (this stream) timed out in its decoupled look-back ",
                    "(a predecessor tile never published); that result is invalid");
    }
}

// Waits for the current stream of `device` and raises if any scan issued on it gave up a look-back.
void scan_check(int64_t device) {
    const at::Device d(at::kCUDA, (c10::DeviceIndex)device);
    const at::DeviceGuard g(d);
    hipStream_t s = c10::hip::getCurrentHIPStream(d.index()).stream();
    TORCH_CHECK(hipStreamSynchronize(s) == hipSuccess, "scan_check: stream synchronize");
    raise_pending_scan_error((int)device, s);
}

at::Tensor scan_out(const at::Tensor& x, at::Tensor out, bool exclusive, const c10::optional<at::Tensor>& init) {
    check_gpu(x, "x", at::kFloat), check_gpu(out, "out", at::kFloat);
    TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.numel() == out.numel(), "scan: contiguous same-size tensors");
    TORCH_CHECK(out.device() == x.device(), "scan: out must be on x's device");
    const at::DeviceGuard g(x.device());
    hipStream_t stream = cur_stream(x);
    unsigned* err_dev = scan_err_word(x.device().index(), stream).dev;
    raise_pending_scan_error(x.device().index(), stream);
    const float* init_ptr = nullptr;
    at::Tensor init_c;
    if (init.has_value() && init->defined()) {
        check_gpu(*init, "init", at::kFloat);
        TORCH_CHECK(init->numel() >= 1 && init->device() == x.device(), "scan: init needs >= 1 element on x's device");
        init_c = init->contiguous();
        init_ptr = init_c.data_ptr<float>();
    }
    at::Tensor xc = x, oc = out;
    if ((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15u) || (reinterpret_cast<uintptr_t>(out.data_ptr()) & 15u)) {
        xc = x.clone();
        oc = at::empty_like(xc);
    }
    auto ws = workspace(x, pcmx_scan_workspace_bytes(xc.numel()));
    check_rc(pcmx_scan_f32(xc.data_ptr<float>(), oc.data_ptr<float>(), xc.numel(), exclusive ? 1 : 0, init_ptr, ws.data_ptr(),
                           err_dev, stream),
             "scan");
    if (!oc.is_same(out)) out.copy_(oc);
    return out;
}

at::Tensor scan(const at::Tensor& x, bool exclusive, const c10::optional<at::Tensor>& init) {
    auto xc = aligned_contig(x).view(-1);
    auto out = at::empty_like(xc);
    return scan_out(xc, out, exclusive, init).view(x.sizes());
}

// ---------------------------------------------------------------- SGEMM
at::Tensor sgemm_out(const at::Tensor& a, const at::Tensor& b, at::Tensor c, double alpha, double beta, int64_t variant) {
    check_gpu(a, "a", at::kFloat), check_gpu(b, "b", at::kFloat), check_gpu(c, "c", at::kFloat);
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "sgemm: 2-D tensors");
    TORCH_CHECK(a.size(1) == b.size(0) && c.size(0) == a.size(0) && c.size(1) == b.size(1), "sgemm: shape mismatch");
    TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && c.stride(1) == 1, "sgemm: row-major operands");
    const at::DeviceGuard g(a.device());
    const int M = (int)a.size(0), N = (int)b.size(1), K = (int)a.size(1);
    int rc;
    if (variant < 0)
        rc = pcmx_sgemm_f32(a.data_ptr<float>(), b.data_ptr<float>(), c.data_ptr<float>(), M, N, K, (int)a.stride(0),
                            (int)b.stride(0), (int)c.stride(0), (float)alpha, (float)beta, cur_stream(a));
    else
        rc = pcmx_sgemm_f32_variant(a.data_ptr<float>(), b.data_ptr<float>(), c.data_ptr<float>(), M, N, K, (int)a.stride(0),
                                    (int)b.stride(0), (int)c.stride(0), (float)alpha, (float)beta, (int)variant, cur_stream(a));
    check_rc(rc, "sgemm (shape must be tile-aligned; use parallel_c_programs_amd.ops.sgemm for any shape)");
    return c;
}

at::Tensor sgemm(const at::Tensor& a, const at::Tensor& b, int64_t variant) {
    auto c = at::empty({a.size(0), b.size(1)}, a.options());
    return sgemm_out(a, b, c, 1.0, 0.0, variant);
}

at::Tensor sgemm_simt(const at::Tensor& a, const at::Tensor& b) {
    check_gpu(a, "a", at::kFloat), check_gpu(b, "b", at::kFloat);
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(0), "sgemm_simt: shape mismatch");
    const at::DeviceGuard g(a.device());
    auto ac = a.contiguous(), bc = b.contiguous();
    auto c = at::empty({a.size(0), b.size(1)}, a.options());
    check_rc(pcmx_sgemm_f32_simt(ac.data_ptr<float>(), bc.data_ptr<float>(), c.data_ptr<float>(), (int)a.size(0), (int)b.size(1),
                                 (int)a.size(1), cur_stream(a)),
             "sgemm_simt");
    return c;
}

void device_info(int64_t device) { pcmx_print_device_info((int)device); }

void check_u8_gpu(const at::Tensor& t, const char* name) {
    check_gpu(t, name, at::kByte);
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// ---------------------------------------------------------------- histogram equalisation
// The multi-block histeq keeps its histogram + ticket in a workspace that every call leaves zeroed, so it is
// allocated (and zeroed) once per (device, stream): no memset launch per call, and calls on different streams
// never share one.
at::Tensor& histeq_workspace(const at::Tensor& like, hipStream_t s) {
    static std::mutex mu;
    static auto* cache = new std::map<std::pair<int, hipStream_t>, at::Tensor>();  // never destroyed: no frees at exit
    std::lock_guard<std::mutex> lock(mu);
    auto& ws = (*cache)[{like.device().index(), s}];
    if (!ws.defined()) ws = at::zeros({pcmx_histeq_workspace_bytes()}, like.options().dtype(at::kByte));
    return ws;
}

at::Tensor histeq(const at::Tensor& img) {
    check_u8_gpu(img, "img");
    const at::DeviceGuard g(img.device());
    auto ic = aligned_contig(img);
    auto out = at::empty_like(ic);
    const hipStream_t s = cur_stream(img);
    auto& ws = histeq_workspace(ic, s);
    const int rc = pcmx_histeq_u8(ic.data_ptr<uint8_t>(), out.data_ptr<uint8_t>(), ic.numel(), ws.data_ptr(), s);
    if (rc) ws.zero_();  // a failed call may leave the self-cleaning replicas/ticket dirty: re-arm before raising
    check_rc(rc, "histeq");
    return out;
}

// ---------------------------------------------------------------- region growing
int64_t region2d_grow_(at::Tensor region, const at::Tensor& img, int64_t thr, int64_t batch, int64_t max_launches) {
    check_u8_gpu(region, "region"), check_u8_gpu(img, "img");
    TORCH_CHECK(region.dim() == 2 && img.sizes() == region.sizes() && region.device() == img.device() &&
                    img.size(0) > 2 && img.size(1) > 2,
                "region2d: padded (H+2, W+2) uint8 tensors on one device");
    const at::DeviceGuard g(img.device());
    const int H = (int)img.size(0) - 2, W = (int)img.size(1) - 2;
    auto ws = workspace(img, pcmx_region2d_workspace_bytes(H, W));
    int launches = 0;
    check_rc(pcmx_region2d_grow(img.data_ptr<uint8_t>(), region.data_ptr<uint8_t>(), H, W, (int)img.size(1), (int)thr,
                                ws.data_ptr(), (int)batch, (int)max_launches, cur_stream(img), &launches),
             "region2d_grow_");
    return launches;
}

int64_t region3d_grow_(at::Tensor region, const at::Tensor& data, int64_t thr, bool tiled, int64_t batch,
                       int64_t max_launches) {
    check_u8_gpu(region, "region"), check_u8_gpu(data, "data");
    TORCH_CHECK(data.dim() == 3 && data.size(0) == data.size(1) && data.size(1) == data.size(2) &&
                    region.sizes() == data.sizes() && region.device() == data.device(),
                "region3d: cubic uint8 volumes on one device");
    const at::DeviceGuard g(data.device());
    const int dim = (int)data.size(0);
    int launches = 0;
    if (tiled) {
        auto ws = workspace(data, pcmx_region3d_workspace_bytes(dim));
        check_rc(pcmx_region3d_grow_tiled(data.data_ptr<uint8_t>(), region.data_ptr<uint8_t>(), dim, (int)thr, ws.data_ptr(),
                                          (int)batch, (int)max_launches, cur_stream(data), &launches),
                 "region3d_grow_ (tiled)");
    } else {
        auto flag = at::empty({4}, data.options().dtype(at::kInt));
        check_rc(pcmx_region3d_grow_naive(data.data_ptr<uint8_t>(), region.data_ptr<uint8_t>(), dim, (int)thr,
                                          flag.data_ptr<int>(), (int)max_launches, cur_stream(data), &launches),
                 "region3d_grow_ (naive)");
    }
    return launches;
}

// z-slab with its halo planes: (nz + 2, dim, dim) uint8 tensors; planes 1..nz are grown, plane 0 / nz + 1 are
// read-only halo seeds when halos bit 0 / bit 1 is set (neighbour ranks' boundary planes)
int64_t region3d_grow_slab_(at::Tensor region, const at::Tensor& data, int64_t halos, int64_t thr, int64_t batch,
                            int64_t max_launches) {
    check_u8_gpu(region, "region"), check_u8_gpu(data, "data");
    TORCH_CHECK(data.dim() == 3 && data.size(1) == data.size(2) && data.size(0) >= 3 && region.sizes() == data.sizes() &&
                    region.device() == data.device(),
                "region3d_grow_slab_: (nz + 2, dim, dim) uint8 slabs with halo planes, on one device");
    TORCH_CHECK(halos >= 0 && halos <= 3, "region3d_grow_slab_: halos in 0..3");
    const at::DeviceGuard g(data.device());
    const int dim = (int)data.size(1), nz = (int)data.size(0) - 2;
    const size_t plane = (size_t)dim * dim;
    auto ws = workspace(data, pcmx_region3d_slab_workspace_bytes(dim, nz));
    int launches = 0;
    check_rc(pcmx_region3d_grow_slab(data.data_ptr<uint8_t>() + plane, region.data_ptr<uint8_t>() + plane, dim, nz,
                                     (int)halos, (int)thr, ws.data_ptr(), (int)batch, (int)max_launches, cur_stream(data),
                                     &launches),
             "region3d_grow_slab_");
    return launches;
}

// ---------------------------------------------------------------- volume + ray casting
void check_cubic(const at::Tensor& v, const char* what) {
    TORCH_CHECK(v.dim() == 3 && v.size(0) == v.size(1) && v.size(1) == v.size(2) && v.size(0) > 1, what,
                ": a cubic (dim, dim, dim) volume with dim > 1");
}

at::Tensor volume_gen_(at::Tensor data, int64_t seed) {
    check_u8_gpu(data, "data");
    check_cubic(data, "volume_gen_");
    const at::DeviceGuard g(data.device());
    check_rc(pcmx_volume_gen_u8(data.data_ptr<uint8_t>(), (int)data.size(0), (unsigned)seed, cur_stream(data)), "volume_gen_");
    return data;
}

at::Tensor volume_gen_slab_(at::Tensor data, int64_t z_first, int64_t seed) {
    check_u8_gpu(data, "data");
    TORCH_CHECK(data.dim() == 3 && data.size(1) == data.size(2) && data.size(0) >= 1,
                "volume_gen_slab_: (nplanes, dim, dim) uint8");
    const at::DeviceGuard g(data.device());
    check_rc(pcmx_volume_gen_slab_u8(data.data_ptr<uint8_t>(), (int)data.size(1), (int)z_first, (int)data.size(0),
                                     (unsigned)seed, cur_stream(data)),
             "volume_gen_slab_");
    return data;
}

std::vector<float> cam_vec(at::ArrayRef<double> cam12) {
    TORCH_CHECK(cam12.size() == 12, "camera: 12 floats (camera, forward, right, up)");
    std::vector<float> c(12);
    for (int i = 0; i < 12; ++i) c[i] = (float)cam12[i];
    return c;
}

at::Tensor raycast_global(const at::Tensor& data, const at::Tensor& region, int64_t image_dim, at::ArrayRef<double> cam12,
                          double pixel_width, double step, int64_t max_steps, bool f64_color, int64_t variant) {
    check_u8_gpu(data, "data"), check_u8_gpu(region, "region");
    check_cubic(data, "raycast_global");
    TORCH_CHECK(region.sizes() == data.sizes() && region.device() == data.device(),
                "raycast_global: region must match data's shape and device");
    TORCH_CHECK(image_dim > 0, "raycast_global: image_dim > 0");
    const at::DeviceGuard g(data.device());
    auto img = at::empty({image_dim, image_dim}, data.options());
    auto c = cam_vec(cam12);
    if (variant < 0) {  // the production rule (pcmx_raycast_global): 16-lane groups, DR16 + 4-lane groups above 2^16 rays
        variant = (image_dim * image_dim > (1 << 16) && data.size(0) % 4 == 0) ? 11 : 6;
    }
    if (variant >= 9) {  // the DR16 layout (data and region interleaved per voxel), packed on this call
        const int dim = (int)data.size(0);
        TORCH_CHECK(dim % 4 == 0, "raycast_global: DR16 variants need dim % 4 == 0");
        auto dr = at::empty({pcmx_raycast_dr16_bytes(dim)}, data.options());
        check_rc(pcmx_raycast_dr16_pack(data.data_ptr<uint8_t>(), region.data_ptr<uint8_t>(), dim, dr.data_ptr(),
                                        cur_stream(data)),
                 "raycast_dr16_pack");
        check_rc(pcmx_raycast_global_dr(dr.data_ptr(), dim, img.data_ptr<uint8_t>(), (int)image_dim, c.data(),
                                        (float)pixel_width, (float)step, (int)max_steps, f64_color ? 1 : 0, (int)variant,
                                        cur_stream(data)),
                 "raycast_global_dr");
        return img;
    }
    check_rc(pcmx_raycast_global_variant(data.data_ptr<uint8_t>(), region.data_ptr<uint8_t>(), (int)data.size(0),
                                         img.data_ptr<uint8_t>(), (int)image_dim, c.data(), (float)pixel_width, (float)step,
                                         (int)max_steps, f64_color ? 1 : 0, (int)variant, cur_stream(data)),
             "raycast_global");
    return img;
}

// slab buffers (nz + 2, dim, dim) starting at global plane z0 - 1; state int32 [image_dim^2, 6]
at::Tensor raycast_slab_(const at::Tensor& data, const at::Tensor& region, int64_t z0, at::Tensor state, bool init,
                         bool bottom, int64_t image_dim, at::ArrayRef<double> cam12, double pixel_width, double step,
                         int64_t max_steps) {
    check_u8_gpu(data, "data"), check_u8_gpu(region, "region");
    check_gpu(state, "state", at::kInt);
    TORCH_CHECK(data.dim() == 3 && data.size(1) == data.size(2) && data.size(0) >= 3 && region.sizes() == data.sizes(),
                "raycast_slab_: (nz + 2, dim, dim) uint8 slabs");
    TORCH_CHECK(state.is_contiguous() && state.numel() == image_dim * image_dim * 6 && state.device() == data.device(),
                "raycast_slab_: state int32 [image_dim^2, 6] on data's device");
    const int dim = (int)data.size(1);
    TORCH_CHECK(z0 >= 0 && z0 + data.size(0) - 2 <= dim, "raycast_slab_: slab planes inside the volume");
    const at::DeviceGuard g(data.device());
    auto img = at::empty({bottom ? image_dim : 0, bottom ? image_dim : 0}, data.options());
    auto c = cam_vec(cam12);
    check_rc(pcmx_raycast_slab(data.data_ptr<uint8_t>(), region.data_ptr<uint8_t>(), dim, (int)z0, state.data_ptr<int>(),
                               init ? 1 : 0, bottom ? 1 : 0, bottom ? img.data_ptr<uint8_t>() : nullptr, (int)image_dim,
                               c.data(), (float)pixel_width, (float)step, (int)max_steps, cur_stream(data)),
             "raycast_slab_");
    return img;
}

at::Tensor brick_pack(const at::Tensor& data, const at::Tensor& region) {
    check_u8_gpu(data, "data"), check_u8_gpu(region, "region");
    const at::DeviceGuard g(data.device());
    TORCH_CHECK(data.dim() == 3 && data.sizes() == region.sizes() && data.size(0) == data.size(1) &&
                    data.size(0) == data.size(2) && data.size(0) <= 2048 && data.is_contiguous() && region.is_contiguous(),
                "brick_pack: contiguous cubic volumes, dim <= 2048");
    auto tex = at::empty({data.numel() * 2 + 2}, data.options().dtype(at::kLong));  // texels + format flag
    check_rc(pcmx_brick_pack(data.data_ptr<uint8_t>(), region.data_ptr<uint8_t>(), (int)data.size(0), tex.data_ptr(),
                             cur_stream(data)),
             "brick_pack");
    return tex;
}

at::Tensor raycast_bricked(const at::Tensor& tex, int64_t image_dim, at::ArrayRef<double> cam12, double pixel_width,
                           double step, int64_t max_steps, int64_t batch, int64_t segments) {
    check_gpu(tex, "tex", at::kLong);
    TORCH_CHECK(tex.dim() == 1 && tex.numel() >= 18 && tex.is_contiguous(), "raycast_bricked: tex from brick_pack");
    const int64_t nvox = (tex.numel() - 2) / 2;
    int64_t dim = (int64_t)std::llround(std::cbrt((double)nvox));
    TORCH_CHECK(dim * dim * dim == nvox, "raycast_bricked: tex from brick_pack of a cubic volume");
    const at::DeviceGuard g(tex.device());
    auto img = at::empty({image_dim, image_dim}, tex.options().dtype(at::kByte));
    auto c = cam_vec(cam12);
    check_rc(pcmx_raycast_bricked(tex.data_ptr(), (int)dim,
                                  img.data_ptr<uint8_t>(), (int)image_dim, c.data(), (float)pixel_width, (float)step,
                                  (int)max_steps, (int)batch, (int)segments, cur_stream(tex)),
             "raycast_bricked");
    return img;
}

// ---------------------------------------------------------------- stencil
void stencil5_(const at::Tensor& u, at::Tensor out, int64_t r0, int64_t r1, int64_t global_row0, int64_t global_rows,
               double k) {
    check_gpu(u, "u", at::kBFloat16), check_gpu(out, "out", at::kBFloat16);
    TORCH_CHECK(u.dim() == 2 && u.sizes() == out.sizes() && u.is_contiguous() && out.is_contiguous(),
                "stencil5: slabs of shape (rows+2, cols)");
    const at::DeviceGuard g(u.device());
    const int rows = (int)u.size(0) - 2, cols = (int)u.size(1);
    check_rc(pcmx_stencil5_bf16(u.data_ptr(), out.data_ptr(), rows, cols, cols, (int)r0, (int)r1, global_row0, global_rows,
                                (float)k, cur_stream(u)),
             "stencil5_");
}

void stencil5xT_(const at::Tensor& u, at::Tensor out, int64_t halo, int64_t steps, int64_t r0, int64_t r1,
                 int64_t global_row0, int64_t global_rows, double k, int64_t shape) {
    check_gpu(u, "u", at::kBFloat16), check_gpu(out, "out", at::kBFloat16);
    TORCH_CHECK(u.dim() == 2 && u.sizes() == out.sizes() && u.is_contiguous() && out.is_contiguous() && halo >= 1 &&
                    u.size(0) > 2 * halo,
                "stencil5xT: slabs of shape (rows + 2*halo, cols)");
    const at::DeviceGuard g(u.device());
    const int rows = (int)(u.size(0) - 2 * halo), cols = (int)u.size(1);
    check_rc(pcmx_stencil5xT_bf16_spans_shape(u.data_ptr(), out.data_ptr(), rows, cols, cols, (int)halo, (int)steps,
                                              (int)r0, (int)r1, 0, 0, global_row0, global_rows, (float)k, (int)shape,
                                              cur_stream(u)),
             "stencil5xT_");
}

void stencil5xT_spans_(const at::Tensor& u, at::Tensor out, int64_t halo, int64_t steps, int64_t r0a, int64_t r1a,
                       int64_t r0b, int64_t r1b, int64_t global_row0, int64_t global_rows, double k, int64_t shape) {
    check_gpu(u, "u", at::kBFloat16), check_gpu(out, "out", at::kBFloat16);
    TORCH_CHECK(u.dim() == 2 && u.sizes() == out.sizes() && u.is_contiguous() && out.is_contiguous() && halo >= 1 &&
                    u.size(0) > 2 * halo,
                "stencil5xT_spans: slabs of shape (rows + 2*halo, cols)");
    const at::DeviceGuard g(u.device());
    const int rows = (int)(u.size(0) - 2 * halo), cols = (int)u.size(1);
    check_rc(pcmx_stencil5xT_bf16_spans_shape(u.data_ptr(), out.data_ptr(), rows, cols, cols, (int)halo, (int)steps,
                                              (int)r0a, (int)r1a, (int)r0b, (int)r1b, global_row0, global_rows, (float)k,
                                              (int)shape, cur_stream(u)),
             "stencil5xT_spans_");
}

// ---------------------------------------------------------------- SpMV
at::Tensor spmv_csr(const at::Tensor& row_ptr, const at::Tensor& col, const at::Tensor& val, const at::Tensor& x,
                    const at::Tensor& items) {
    check_gpu(row_ptr, "row_ptr", at::kLong), check_gpu(col, "col", at::kInt), check_gpu(val, "val", at::kFloat);
    check_gpu(x, "x", at::kFloat), check_gpu(items, "items", at::kLong);
    const at::DeviceGuard g(val.device());
    const int n_rows = (int)row_ptr.numel() - 1;
    auto y = at::empty({n_rows}, val.options());
    check_rc(pcmx_spmv_csr((const long long*)row_ptr.data_ptr<int64_t>(), col.data_ptr<int>(), val.data_ptr<float>(), x.data_ptr<float>(),
                           y.data_ptr<float>(), n_rows, items.data_ptr(), items.size(0), cur_stream(val)),
             "spmv_csr");
    return y;
}

// XCD-sliced CSR (see spmv.hip): meta is a CPU int64 tensor [2 * n_slices + 1] = slice nz0[n_slices] ++
// slice item0[n_slices + 1]; ypart [n_slices * n_rows] and extra [n_items] are caller-owned scratch.
at::Tensor spmv_sliced(const at::Tensor& lrow, const at::Tensor& col, const at::Tensor& val, const at::Tensor& x,
                       const at::Tensor& items, const at::Tensor& row_mask, const at::Tensor& chunk_base,
                       const at::Tensor& fix, const at::Tensor& meta, at::Tensor ypart, at::Tensor extra, int64_t n_rows,
                       const c10::optional<at::Tensor>& out, int64_t mode) {
    check_gpu(lrow, "lrow", at::kShort), check_gpu(col, "col", at::kInt), check_gpu(val, "val", at::kFloat);
    check_gpu(x, "x", at::kFloat), check_gpu(items, "items", at::kLong), check_gpu(fix, "fix", at::kInt);
    check_gpu(ypart, "ypart", at::kFloat), check_gpu(extra, "extra", at::kFloat);
    check_gpu(row_mask, "row_mask", at::kInt), check_gpu(chunk_base, "chunk_base", at::kInt);
    TORCH_CHECK(!meta.is_cuda() && meta.scalar_type() == at::kLong && meta.is_contiguous(), "spmv_sliced: CPU int64 meta");
    // mode bit 3: packed layout (col holds one word per nonzero: column offset + head flag + row offset; lrow unused)
    // and meta = [nz0 (S) | item0 (S + 1) | out0 (S + 1) | colbase (S)]; otherwise meta = [nz0 | item0 | out0]
    const bool packed = (mode & 8) != 0;
    const int64_t S = (meta.numel() - 2) / (packed ? 4 : 3);
    TORCH_CHECK(meta.numel() == (packed ? 4 : 3) * S + 2 && S >= 8 && S % 8 == 0 && S <= PCMX_SPMV_MAX_SLICES,
                "spmv_sliced: 8, 16, 24 or 32 slices");
    const int64_t* m = meta.data_ptr<int64_t>();
    const int64_t* out0 = m + 2 * S + 1;
    TORCH_CHECK((packed || lrow.numel() == col.numel()) && val.numel() == col.numel(), "spmv_sliced: lrow / val shape");
    std::vector<int> colbase;
    if (packed) {
        for (int64_t k = 0; k < S; ++k) {
            TORCH_CHECK(m[3 * S + 2 + k] >= 0 && m[3 * S + 2 + k] < x.numel(), "spmv_sliced: packed column base");
            colbase.push_back((int)m[3 * S + 2 + k]);
        }
        TORCH_CHECK((mode & 7) == 0 || (mode & 7) == 2, "spmv_sliced: the packed layout runs the production modes only");
    } else {
        TORCH_CHECK(!(mode & ((1 << 27) | (1 << 28))), "spmv_sliced: 256 / 384-nonzero items need the packed layout");
    }
    TORCH_CHECK(row_mask.numel() >= n_rows && chunk_base.numel() >= ((n_rows + 63) / 64) * S,
                "spmv_sliced: row_mask / chunk_base shape");
    TORCH_CHECK(out0[0] == 0 && ypart.numel() >= out0[S], "spmv_sliced: ypart must hold every compact partial");
    TORCH_CHECK(x.numel() < (int64_t(1) << 30), "spmv_sliced: x must be < 2^30 elements (32-bit buffer offsets)");
    TORCH_CHECK(m[S] >= 0 && m[2 * S] <= items.size(0) && extra.numel() >= items.size(0), "spmv_sliced: items/extra shape");
    TORCH_CHECK(fix.dim() == 2 && fix.size(1) == 2, "spmv_sliced: fix [k, 2]");
    for (int64_t k = 0; k < S; ++k)
        TORCH_CHECK(m[k] >= 0 && m[k] <= col.numel() && m[S + k] <= m[S + k + 1] && out0[k] <= out0[k + 1],
                    "spmv_sliced: meta");
    const at::DeviceGuard g(val.device());
    at::Tensor y;
    if (out.has_value()) {
        y = *out;
        check_gpu(y, "out", at::kFloat);
        TORCH_CHECK(y.is_contiguous() && y.numel() >= n_rows && y.device() == val.device(),
                    "spmv_sliced: out must be a contiguous float32 tensor of >= n_rows elements on val's device");
    } else {
        y = at::empty({n_rows}, val.options());
    }
    check_rc(pcmx_spmv_sliced(reinterpret_cast<const unsigned short*>(lrow.numel() ? lrow.data_ptr<int16_t>() : nullptr),
                              col.data_ptr<int>(),
                              val.data_ptr<float>(), x.data_ptr<float>(), ypart.data_ptr<float>(), extra.data_ptr<float>(),
                              y.data_ptr<float>(), (int)n_rows, (int)x.numel(), (int)S, (const long long*)m,
                              (const long long*)m + S, (const long long*)out0, items.data_ptr(),
                              reinterpret_cast<const unsigned*>(row_mask.data_ptr<int>()), chunk_base.data_ptr<int>(),
                              fix.data_ptr(), (int)fix.size(0), (int)(mode & ~8), packed ? colbase.data() : nullptr,
                              cur_stream(val)),
             "spmv_sliced");
    return y;
}

// Products only of phases [a_lo, a_lo + a_n) of sliced matrix A and [b_lo, b_lo + b_n) of B (same x), ONE launch
// (pcmx_spmv_sliced_pair). meta_*: the packed spmv_sliced meta (nz0 S | item0 S + 1 | out0 S + 1 | colbase S).
void spmv_sliced_pair(const at::Tensor& x, int64_t item_mode, int64_t mode, const at::Tensor& col_a,
                      const at::Tensor& val_a, const at::Tensor& items_a, const at::Tensor& meta_a, at::Tensor ypart_a,
                      at::Tensor extra_a, int64_t s_a, int64_t a_lo, int64_t a_n, const at::Tensor& col_b,
                      const at::Tensor& val_b, const at::Tensor& items_b, const at::Tensor& meta_b, at::Tensor ypart_b,
                      at::Tensor extra_b, int64_t s_b, int64_t b_lo, int64_t b_n) {
    check_gpu(x, "x", at::kFloat);
    TORCH_CHECK(x.numel() < (int64_t(1) << 30), "spmv_sliced_pair: x must be < 2^30 elements");
    auto chk = [&](const at::Tensor& col, const at::Tensor& val, const at::Tensor& items, const at::Tensor& meta,
                   const at::Tensor& ypart, const at::Tensor& extra, int64_t S, int64_t lo, int64_t n) {
        check_gpu(col, "col", at::kInt), check_gpu(val, "val", at::kFloat), check_gpu(items, "items", at::kLong);
        check_gpu(ypart, "ypart", at::kFloat), check_gpu(extra, "extra", at::kFloat);
        TORCH_CHECK(col.device() == x.device() && val.numel() == col.numel(), "spmv_sliced_pair: col / val");
        TORCH_CHECK(S >= 8 && S % 8 == 0 && S <= PCMX_SPMV_MAX_SLICES && lo >= 0 && n >= 0 && 8 * (lo + n) <= S,
                    "spmv_sliced_pair: slices / phases");
        TORCH_CHECK(!meta.is_cuda() && meta.scalar_type() == at::kLong && meta.is_contiguous() && meta.numel() == 4 * S + 2,
                    "spmv_sliced_pair: packed CPU int64 meta");
        const int64_t* m = meta.data_ptr<int64_t>();
        const int64_t* out0 = m + 2 * S + 1;
        TORCH_CHECK(out0[0] == 0 && ypart.numel() >= out0[S] && m[2 * S] <= items.size(0) && extra.numel() >= items.size(0),
                    "spmv_sliced_pair: ypart / items / extra shape");
        for (int64_t k = 0; k < S; ++k)
            TORCH_CHECK(m[k] >= 0 && m[k] <= col.numel() && m[S + k] <= m[S + k + 1] && m[3 * S + 2 + k] >= 0 &&
                            m[3 * S + 2 + k] < x.numel(),
                        "spmv_sliced_pair: meta");
    };
    chk(col_a, val_a, items_a, meta_a, ypart_a, extra_a, s_a, a_lo, a_n);
    chk(col_b, val_b, items_b, meta_b, ypart_b, extra_b, s_b, b_lo, b_n);
    TORCH_CHECK(8 * (a_n + b_n) <= PCMX_SPMV_MAX_SLICES, "spmv_sliced_pair: at most 32 slices per launch");
    auto cb = [](const at::Tensor& meta, int64_t S) {
        std::vector<int> v(S);
        for (int64_t k = 0; k < S; ++k) v[k] = (int)meta.data_ptr<int64_t>()[3 * S + 2 + k];
        return v;
    };
    const auto cba = cb(meta_a, s_a), cbb = cb(meta_b, s_b);
    const int64_t *ma = meta_a.data_ptr<int64_t>(), *mb = meta_b.data_ptr<int64_t>();
    const at::DeviceGuard g(x.device());
    check_rc(pcmx_spmv_sliced_pair(x.data_ptr<float>(), (int)x.numel(), (int)item_mode, (int)mode, col_a.data_ptr<int>(),
                                   val_a.data_ptr<float>(), items_a.data_ptr(), ypart_a.data_ptr<float>(),
                                   extra_a.data_ptr<float>(), (int)s_a, (const long long*)ma, (const long long*)ma + s_a,
                                   (const long long*)ma + 2 * s_a + 1, cba.data(), (int)a_lo, (int)a_n,
                                   col_b.data_ptr<int>(), val_b.data_ptr<float>(), items_b.data_ptr(),
                                   ypart_b.data_ptr<float>(), extra_b.data_ptr<float>(), (int)s_b, (const long long*)mb,
                                   (const long long*)mb + s_b, (const long long*)mb + 2 * s_b + 1, cbb.data(), (int)b_lo,
                                   (int)b_n, cur_stream(x)),
             "spmv_sliced_pair");
}

// The combine + fix-up (+ send-buffer pack) of the partials a products-only spmv_sliced call (mode bit 4) wrote, in one
// launch (pcmx_spmv_sliced_combine). meta: the spmv_sliced meta of the same matrix (out0 at [2S + 1, 3S + 2)).
void spmv_sliced_combine(const at::Tensor& ypart, const at::Tensor& row_mask, const at::Tensor& chunk_base,
                         const at::Tensor& meta, int64_t n_slices, const at::Tensor& extra, const at::Tensor& fix,
                         const c10::optional<at::Tensor>& fix_chunk0, at::Tensor out, int64_t n_rows,
                         const c10::optional<at::Tensor>& send_ptr, const c10::optional<at::Tensor>& send_slot,
                         const c10::optional<at::Tensor>& sendbuf) {
    check_gpu(ypart, "ypart", at::kFloat), check_gpu(extra, "extra", at::kFloat), check_gpu(fix, "fix", at::kInt);
    check_gpu(row_mask, "row_mask", at::kInt), check_gpu(chunk_base, "chunk_base", at::kInt);
    check_gpu(out, "out", at::kFloat);
    const int64_t S = n_slices;
    TORCH_CHECK(S >= 8 && S % 8 == 0 && S <= PCMX_SPMV_MAX_SLICES, "spmv_sliced_combine: 8, 16, 24 or 32 slices");
    TORCH_CHECK(!meta.is_cuda() && meta.scalar_type() == at::kLong && meta.is_contiguous() && meta.numel() >= 3 * S + 2,
                "spmv_sliced_combine: CPU int64 meta");
    const int64_t* out0 = meta.data_ptr<int64_t>() + 2 * S + 1;
    const int64_t chunks = (n_rows + 63) / 64;
    TORCH_CHECK(row_mask.numel() >= n_rows && chunk_base.numel() >= chunks * S, "spmv_sliced_combine: row_mask / chunk_base");
    TORCH_CHECK(out0[0] == 0 && ypart.numel() >= out0[S], "spmv_sliced_combine: ypart must hold every compact partial");
    TORCH_CHECK(out.is_contiguous() && out.numel() >= n_rows && out.device() == ypart.device(), "spmv_sliced_combine: out");
    TORCH_CHECK(fix.dim() == 2 && fix.size(1) == 2, "spmv_sliced_combine: fix [k, 2]");
    const int* fc = nullptr;
    if (fix_chunk0.has_value() && fix.size(0) > 0) {
        check_gpu(*fix_chunk0, "fix_chunk0", at::kInt);
        TORCH_CHECK(fix_chunk0->is_contiguous() && fix_chunk0->numel() >= chunks + 1, "spmv_sliced_combine: fix_chunk0");
        fc = fix_chunk0->data_ptr<int>();
    } else {
        TORCH_CHECK(fix.size(0) == 0, "spmv_sliced_combine: split rows need fix_chunk0");
    }
    const int *sp = nullptr, *ss = nullptr;
    float* sb = nullptr;
    if (send_ptr.has_value()) {
        // INTERNAL op: the list CONTENTS (send_ptr rising from 0 to send_slot.numel(), every slot inside sendbuf) are
        // device data; checking them here would sync every call, so SlicedCSR._check_send (the only caller,
        // ops/sparse.py) validates each set of lists once. Shapes and dtypes are checked here.
        TORCH_CHECK(send_slot.has_value() && sendbuf.has_value(), "spmv_sliced_combine: send_ptr needs send_slot and sendbuf");
        check_gpu(*send_ptr, "send_ptr", at::kInt), check_gpu(*send_slot, "send_slot", at::kInt);
        check_gpu(*sendbuf, "sendbuf", at::kFloat);
        TORCH_CHECK(send_ptr->is_contiguous() && send_ptr->numel() >= n_rows + 1 && send_slot->is_contiguous() &&
                        sendbuf->is_contiguous() && send_slot->numel() <= sendbuf->numel(),
                    "spmv_sliced_combine: send lists");
        if (send_slot->numel() > 0)  // (no peer references any row, e.g. one rank: nothing to pack)
            sp = send_ptr->data_ptr<int>(), ss = send_slot->data_ptr<int>(), sb = sendbuf->data_ptr<float>();
    }
    const at::DeviceGuard g(ypart.device());
    check_rc(pcmx_spmv_sliced_combine(ypart.data_ptr<float>(), reinterpret_cast<const unsigned*>(row_mask.data_ptr<int>()),
                                      chunk_base.data_ptr<int>(), (const long long*)out0, (int)S, out.data_ptr<float>(),
                                      (int)n_rows, extra.data_ptr<float>(), fix.data_ptr(), fc, sp, ss, sb,
                                      cur_stream(ypart)),
             "spmv_sliced_combine");
}

at::Tensor spmv_banded(const at::Tensor& vals, const at::Tensor& row_off, int64_t n, int64_t a, int64_t b, int64_t c,
                       int64_t d, int64_t e, const at::Tensor& x, int64_t variant) {
    check_gpu(vals, "vals", at::kFloat), check_gpu(row_off, "row_off", at::kLong), check_gpu(x, "x", at::kFloat);
    TORCH_CHECK(vals.is_contiguous() && row_off.is_contiguous() && x.is_contiguous(), "spmv_banded: contiguous tensors");
    TORCH_CHECK(row_off.numel() >= n && x.numel() >= n, "spmv_banded: row_off and x need n entries");
    const at::DeviceGuard g(vals.device());
    auto y = at::empty({n}, vals.options());
    check_rc(pcmx_spmv_banded_variant(vals.data_ptr<float>(), (const long long*)row_off.data_ptr<int64_t>(), (int)n, (int)a,
                                      (int)b, (int)c, (int)d, (int)e, x.data_ptr<float>(), y.data_ptr<float>(), (int)variant,
                                      cur_stream(vals)),
             "spmv_banded");
    return y;
}

// ---------------------------------------------------------------- halo pack/unpack
at::Tensor pack_edges(const at::Tensor& tile) {
    TORCH_CHECK(tile.is_cuda() && tile.dim() == 2 && tile.is_contiguous(), "pack_edges: contiguous padded 2-D GPU tile");
    const at::DeviceGuard g(tile.device());
    const int H = (int)tile.size(0) - 2, W = (int)tile.size(1) - 2;
    auto buf = at::empty({2 * W + 2 * H}, tile.options());
    check_rc(pcmx_pack_edges(tile.data_ptr(), (int)tile.element_size(), H, W, (int)tile.size(1), buf.data_ptr(), cur_stream(tile)),
             "pack_edges");
    return buf;
}

void unpack_halo_(at::Tensor tile, const at::Tensor& buf, int64_t mask, const c10::optional<at::Tensor>& changed) {
    TORCH_CHECK(tile.is_cuda() && tile.dim() == 2 && tile.is_contiguous() && buf.dtype() == tile.dtype(), "unpack_halo_");
    TORCH_CHECK(buf.is_cuda() && buf.is_contiguous() && buf.device() == tile.device(), "unpack_halo_: buf on tile's device");
    const at::DeviceGuard g(tile.device());
    const int H = (int)tile.size(0) - 2, W = (int)tile.size(1) - 2;
    TORCH_CHECK(buf.numel() == 2 * W + 2 * H, "unpack_halo_: buffer size");
    int* flag = nullptr;
    if (changed.has_value()) {
        check_gpu(*changed, "changed", at::kInt);
        TORCH_CHECK(changed->numel() >= 1 && changed->device() == tile.device(), "unpack_halo_: changed flag");
        flag = changed->data_ptr<int>();
    }
    check_rc(pcmx_unpack_halo_changed(tile.data_ptr(), (int)tile.element_size(), H, W, (int)tile.size(1), buf.data_ptr(),
                                      (int)mask, flag, cur_stream(tile)),
             "unpack_halo_");
}

// host-side CSR analysis (CPU int64 row_ptr -> int64 [n_items, 3] work items)
at::Tensor spmv_csr_plan(const at::Tensor& row_ptr, int64_t item_nnz) {
    TORCH_CHECK(!row_ptr.is_cuda() && row_ptr.scalar_type() == at::kLong, "spmv_csr_plan: CPU int64 row_ptr");
    auto rp = row_ptr.contiguous();
    const int n_rows = (int)rp.numel() - 1;
    const long long k = pcmx_spmv_csr_plan_nnz((const long long*)rp.data_ptr<int64_t>(), n_rows, nullptr, 0, (int)item_nnz);
    TORCH_CHECK(k >= 0, "spmv_csr_plan: item_nnz must be a multiple of 64 in [64, 1024]");
    auto items = at::empty({k, 3}, rp.options());
    pcmx_spmv_csr_plan_nnz((const long long*)rp.data_ptr<int64_t>(), n_rows, items.data_ptr(), k, (int)item_nnz);
    return items;
}

}  // namespace

TORCH_LIBRARY(pcmx, m) {
    m.def("vmul(Tensor a, Tensor b) -> Tensor");
    m.def("vadd(Tensor a, Tensor b) -> Tensor");
    m.def("axpy_(Tensor(a!) y, float alpha, Tensor x) -> Tensor(a!)");
    m.def("gather_(Tensor src, Tensor idx, Tensor(a!) out) -> Tensor(a!)");
    m.def("fill_(Tensor(a!) x, float v) -> Tensor(a!)");
    m.def("copy_(Tensor(a!) dst, Tensor src) -> Tensor(a!)");
    m.def("rand_uniform_(Tensor(a!) x, int seed, float lo, float hi) -> Tensor(a!)");
    m.def("reduce(Tensor x, int op) -> Tensor");
    m.def("dot(Tensor a, Tensor b) -> Tensor");
    m.def("scan(Tensor x, bool exclusive=False, Tensor? init=None) -> Tensor");
    m.def("scan_out(Tensor x, Tensor(a!) out, bool exclusive=False, Tensor? init=None) -> Tensor(a!)");
    m.def("scan_check(int device=0) -> ()", scan_check);
    m.def("sgemm(Tensor a, Tensor b, int variant=-1) -> Tensor");
    m.def("sgemm_out(Tensor a, Tensor b, Tensor(a!) c, float alpha=1., float beta=0., int variant=-1) -> Tensor(a!)");
    m.def("sgemm_simt(Tensor a, Tensor b) -> Tensor");
    m.def("device_info(int device=0) -> ()", device_info);
    m.def("histeq(Tensor img) -> Tensor");
    m.def("region2d_grow_(Tensor(a!) region, Tensor img, int thr, int batch=4, int max_launches=100000) -> int");
    m.def("region3d_grow_(Tensor(a!) region, Tensor data, int thr, bool tiled=True, int batch=8, int max_launches=1000000) -> int");
    m.def("region3d_grow_slab_(Tensor(a!) region, Tensor data, int halos, int thr, int batch=8, int max_launches=1000000) -> int");
    m.def("volume_gen_(Tensor(a!) data, int seed) -> Tensor(a!)");
    m.def("volume_gen_slab_(Tensor(a!) data, int z_first, int seed) -> Tensor(a!)");
    m.def("raycast_slab_(Tensor data, Tensor region, int z0, Tensor(a!) state, bool init, bool bottom, int image_dim, float[] cam12, float pixel_width, float step, int max_steps) -> Tensor");
    m.def("raycast_global(Tensor data, Tensor region, int image_dim, float[] cam12, float pixel_width, float step, int max_steps, bool f64_color=True, int variant=-1) -> Tensor");
    m.def("brick_pack(Tensor data, Tensor region) -> Tensor");
    m.def("raycast_bricked(Tensor tex, int image_dim, float[] cam12, float pixel_width, float step, int max_steps, int batch=0, int segments=0) -> Tensor");
    m.def("stencil5_(Tensor u, Tensor(a!) out, int r0, int r1, int global_row0, int global_rows, float k) -> ()");
    m.def("stencil5xT_(Tensor u, Tensor(a!) out, int halo, int steps, int r0, int r1, int global_row0, int global_rows, float k, int shape=0) -> ()");
    m.def("stencil5xT_spans_(Tensor u, Tensor(a!) out, int halo, int steps, int r0a, int r1a, int r0b, int r1b, int global_row0, int global_rows, float k, int shape=0) -> ()");
    m.def("spmv_csr(Tensor row_ptr, Tensor col, Tensor val, Tensor x, Tensor items) -> Tensor");
    m.def("spmv_sliced(Tensor lrow, Tensor col, Tensor val, Tensor x, Tensor items, Tensor row_mask, Tensor chunk_base, Tensor fix, Tensor meta, Tensor(a!) ypart, Tensor(b!) extra, int n_rows, Tensor(c!)? out=None, int mode=0) -> Tensor");
    m.def("spmv_sliced_pair(Tensor x, int item_mode, int mode, Tensor col_a, Tensor val_a, Tensor items_a, Tensor meta_a, Tensor(a!) ypart_a, Tensor(b!) extra_a, int s_a, int a_lo, int a_n, Tensor col_b, Tensor val_b, Tensor items_b, Tensor meta_b, Tensor(c!) ypart_b, Tensor(d!) extra_b, int s_b, int b_lo, int b_n) -> ()");
    m.def("spmv_sliced_combine(Tensor ypart, Tensor row_mask, Tensor chunk_base, Tensor meta, int n_slices, Tensor extra, Tensor fix, Tensor? fix_chunk0, Tensor(a!) out, int n_rows, Tensor? send_ptr=None, Tensor? send_slot=None, Tensor(b!)? sendbuf=None) -> ()");
    m.def("spmv_banded(Tensor vals, Tensor row_off, int n, int a, int b, int c, int d, int e, Tensor x, int variant=8) -> Tensor");
    m.def("pack_edges(Tensor tile) -> Tensor");
    m.def("unpack_halo_(Tensor(a!) tile, Tensor buf, int mask, Tensor(b!)? changed=None) -> ()");
}

TORCH_LIBRARY_IMPL(pcmx, CUDA, m) {
    m.impl("vmul", vmul);
    m.impl("vadd", vadd);
    m.impl("axpy_", axpy_);
    m.impl("gather_", gather_);
    m.impl("fill_", fill_);
    m.impl("copy_", copy_);
    m.impl("rand_uniform_", rand_uniform_);
    m.impl("reduce", reduce);
    m.impl("dot", dot);
    m.impl("scan", scan);
    m.impl("scan_out", scan_out);
    m.impl("sgemm", sgemm);
    m.impl("sgemm_out", sgemm_out);
    m.impl("sgemm_simt", sgemm_simt);
    m.impl("histeq", histeq);
    m.impl("region2d_grow_", region2d_grow_);
    m.impl("region3d_grow_", region3d_grow_);
    m.impl("volume_gen_", volume_gen_);
    m.impl("raycast_global", raycast_global);
    m.impl("brick_pack", brick_pack);
    m.impl("raycast_bricked", raycast_bricked);
    m.impl("region3d_grow_slab_", region3d_grow_slab_);
    m.impl("volume_gen_slab_", volume_gen_slab_);
    m.impl("raycast_slab_", raycast_slab_);
    m.impl("stencil5_", stencil5_);
    m.impl("stencil5xT_", stencil5xT_);
    m.impl("stencil5xT_spans_", stencil5xT_spans_);
    m.impl("spmv_csr", spmv_csr);
    m.impl("spmv_sliced", spmv_sliced);
    m.impl("spmv_sliced_pair", spmv_sliced_pair);
    m.impl("spmv_sliced_combine", spmv_sliced_combine);
    m.impl("spmv_banded", spmv_banded);
    m.impl("pack_edges", pack_edges);
    m.impl("unpack_halo_", unpack_halo_);
}

// ---------------------------------------------------------------- grouped exchange (dedicated RCCL communicator)
// Plain pybind functions (no torch dispatcher on the per-step path): parallel/dist.py NativeExchange.
pybind11::bytes xcomm_unique_id() {
    std::string id((size_t)pcmx_xcomm_id_bytes(), '\0');
    check_rc(pcmx_xcomm_unique_id(id.data()), "xcomm_unique_id");
    return pybind11::bytes(id);
}

int64_t xcomm_create(const std::string& id, int64_t world, int64_t rank, int64_t device) {
    TORCH_CHECK((int)id.size() == pcmx_xcomm_id_bytes(), "xcomm_create: unique id of ", pcmx_xcomm_id_bytes(), " bytes");
    void* h = nullptr;
    check_rc(pcmx_xcomm_create(id.data(), (int)world, (int)rank, (int)device, &h), "xcomm_create");
    return reinterpret_cast<int64_t>(h);
}

void xcomm_exchange(int64_t h, int64_t slot, const at::Tensor& send, const std::vector<int64_t>& soff,
                    const std::vector<int64_t>& scnt, at::Tensor recv, const std::vector<int64_t>& roff,
                    const std::vector<int64_t>& rcnt) {
    TORCH_CHECK(send.is_cuda() && recv.is_cuda() && send.device() == recv.device(), "xcomm_exchange: GPU buffers, one device");
    TORCH_CHECK(send.is_contiguous() && recv.is_contiguous() && send.scalar_type() == recv.scalar_type(),
                "xcomm_exchange: contiguous buffers of one dtype");
    const size_t W = soff.size();
    TORCH_CHECK(W > 0 && scnt.size() == W && roff.size() == W && rcnt.size() == W, "xcomm_exchange: one entry per rank");
    const int64_t es = send.element_size();
    std::vector<int64_t> b(4 * W);  // the segments in bytes
    for (size_t q = 0; q < W; ++q) {  // every segment inside its buffer (host-side, no device data involved)
        TORCH_CHECK(scnt[q] >= 0 && soff[q] >= 0 && soff[q] + scnt[q] <= send.numel(), "xcomm_exchange: send segment ", q);
        TORCH_CHECK(rcnt[q] >= 0 && roff[q] >= 0 && roff[q] + rcnt[q] <= recv.numel(), "xcomm_exchange: recv segment ", q);
        b[q] = soff[q] * es, b[W + q] = scnt[q] * es, b[2 * W + q] = roff[q] * es, b[3 * W + q] = rcnt[q] * es;
    }
    const auto* bl = reinterpret_cast<const long long*>(b.data());
    check_rc(pcmx_xcomm_exchange(reinterpret_cast<void*>(h), (int)slot, send.data_ptr(), bl, bl + W, recv.data_ptr(),
                                 bl + 2 * W, bl + 3 * W, cur_stream(recv)),
             "xcomm_exchange");
}

void xcomm_wait(int64_t h, int64_t slot, int64_t device) {
    check_rc(pcmx_xcomm_wait(reinterpret_cast<void*>(h), (int)slot, c10::hip::getCurrentHIPStream((int)device).stream()),
             "xcomm_wait");
}

PYBIND11_MODULE(_C, mod) {
    mod.doc() = "pcmx MI355X kernels (ops live under torch.ops.pcmx)";
    mod.def("device_count", []() { return pcmx_device_count(); });
    mod.def("spmv_csr_plan", &spmv_csr_plan, "CSR-adaptive work items from a CPU int64 row_ptr",
            pybind11::arg("row_ptr"), pybind11::arg("item_nnz") = 1024);
    mod.def("xcomm_unique_id", &xcomm_unique_id, "ncclUniqueId of a new dedicated RCCL communicator (rank 0)");
    mod.def("xcomm_create", &xcomm_create, "join the dedicated RCCL communicator: handle");
    mod.def("xcomm_exchange", &xcomm_exchange, "grouped per-peer send/recv of float segments, ordered after the "
            "current stream (slot: one exchange in flight)");
    mod.def("xcomm_wait", &xcomm_wait, "the current stream of `device` waits for the slot's exchange");
    mod.def("xcomm_probe", [](int64_t h, int64_t timeout_ms) {
        pybind11::gil_scoped_release nogil;
        return pcmx_xcomm_probe(reinterpret_cast<void*>(h), (int)timeout_ms);
    }, "one float to / from every peer, host-waited with a timeout; aborts the communicator on failure (0: ok)");
    mod.def("xcomm_async_error", [](int64_t h) { return pcmx_xcomm_async_error(reinterpret_cast<void*>(h)); });
    mod.def("xcomm_destroy", [](int64_t h) { return pcmx_xcomm_destroy(reinterpret_cast<void*>(h)); });
}
