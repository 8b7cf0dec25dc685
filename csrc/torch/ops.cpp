// Torch op registrations: every MI355X kernel of libpcmx_hip.so is exposed as torch.ops.pcmx.<name>.
// GPU tensors dispatch here (DispatchKey "CUDA" is the HIP device on ROCm builds of PyTorch); kernels
// run on the current torch HIP stream so they compose with torch.distributed (RCCL) streams and hipGraph
// capture. Workspaces come from the torch caching allocator (no hipMalloc on the launch path).
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

at::Tensor axpy_(at::Tensor y, double alpha, const at::Tensor& x) {
    check_gpu(y, "y", at::kFloat), check_gpu(x, "x", at::kFloat);
    TORCH_CHECK(y.is_contiguous() && (reinterpret_cast<uintptr_t>(y.data_ptr()) & 15u) == 0, "axpy_: y must be contiguous, 16-B aligned");
    TORCH_CHECK(x.numel() == y.numel(), "axpy_: size mismatch");
    const at::DeviceGuard g(y.device());
    auto xc = aligned_contig(x);
    check_rc(pcmx_axpy_f32((float)alpha, xc.data_ptr<float>(), y.data_ptr<float>(), y.numel(), cur_stream(y)), "axpy_");
    return y;
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

at::Tensor scan_out(const at::Tensor& x, at::Tensor out, bool exclusive, const c10::optional<at::Tensor>& init) {
    check_gpu(x, "x", at::kFloat), check_gpu(out, "out", at::kFloat);
    TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.numel() == out.numel(), "scan: contiguous same-size tensors");
    const at::DeviceGuard g(x.device());
    const float* init_ptr = nullptr;
    at::Tensor init_c;
    if (init.has_value() && init->defined()) {
        check_gpu(*init, "init", at::kFloat);
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
                           cur_stream(x)),
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

}  // namespace

TORCH_LIBRARY(pcmx, m) {
    m.def("vmul(Tensor a, Tensor b) -> Tensor");
    m.def("vadd(Tensor a, Tensor b) -> Tensor");
    m.def("axpy_(Tensor(a!) y, float alpha, Tensor x) -> Tensor(a!)");
    m.def("fill_(Tensor(a!) x, float v) -> Tensor(a!)");
    m.def("rand_uniform_(Tensor(a!) x, int seed, float lo, float hi) -> Tensor(a!)");
    m.def("reduce(Tensor x, int op) -> Tensor");
    m.def("dot(Tensor a, Tensor b) -> Tensor");
    m.def("scan(Tensor x, bool exclusive=False, Tensor? init=None) -> Tensor");
    m.def("scan_out(Tensor x, Tensor(a!) out, bool exclusive=False, Tensor? init=None) -> Tensor(a!)");
    m.def("sgemm(Tensor a, Tensor b, int variant=-1) -> Tensor");
    m.def("sgemm_out(Tensor a, Tensor b, Tensor(a!) c, float alpha=1., float beta=0., int variant=-1) -> Tensor(a!)");
    m.def("sgemm_simt(Tensor a, Tensor b) -> Tensor");
    m.def("device_info(int device=0) -> ()", device_info);
}

TORCH_LIBRARY_IMPL(pcmx, CUDA, m) {
    m.impl("vmul", vmul);
    m.impl("vadd", vadd);
    m.impl("axpy_", axpy_);
    m.impl("fill_", fill_);
    m.impl("rand_uniform_", rand_uniform_);
    m.impl("reduce", reduce);
    m.impl("dot", dot);
    m.impl("scan", scan);
    m.impl("scan_out", scan_out);
    m.impl("sgemm", sgemm);
    m.impl("sgemm_out", sgemm_out);
    m.impl("sgemm_simt", sgemm_simt);
}

PYBIND11_MODULE(_C, mod) {
    mod.doc() = "pcmx MI355X kernels (ops live under torch.ops.pcmx)";
    mod.def("device_count", []() { return pcmx_device_count(); });
}
