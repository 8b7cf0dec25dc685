// Element-wise streaming kernels (HBM-bound): vmul (ref 6-opencl-region-growing/multiply_opencl.cl:1-4),
// vadd/axpy (north-star vector-add), fill and on-device uniform random generation.
//
// MI355X design: 16-B (f32x4) accesses per lane so one wave instruction moves 1 KiB, 4 independent
// f32x4 per lane per iteration to keep enough bytes in flight, non-temporal hints on streamed-once
// data, grid capped at 256 CUs x 64 blocks with a grid-stride loop (cdna_hip_programming.md G11/G13; the write side
// of an HBM stream tops out near 5.5 TB/s on MI355X: vadd 1e9 2.18 ms = 5.5 TB/s, fill 5.6, against 7.1 for a
// read-only stream, profiles/r4_bench/stream_bw_lab.txt).
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
using pcmx::kWave;
constexpr int kThreads = 256;
constexpr int kUnroll = 4;

using pcmx::f32x4;
using pcmx::ld_nt;
using pcmx::st_nt;

template <class F>
__device__ __forceinline__ void stream_binary(const float* a, const float* b, float* r, long long n, F f) {
    const long long n4 = n >> 2;
    const f32x4* a4 = reinterpret_cast<const f32x4*>(a);
    const f32x4* b4 = reinterpret_cast<const f32x4*>(b);
    f32x4* r4 = reinterpret_cast<f32x4*>(r);
    const long long stride = (long long)gridDim.x * kThreads;
    long long i = (long long)blockIdx.x * kThreads * kUnroll + threadIdx.x;
    for (; i + (kUnroll - 1) * kThreads < n4; i += stride * kUnroll) {
        f32x4 va[kUnroll], vb[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) va[u] = ld_nt(a4 + i + u * kThreads), vb[u] = ld_nt(b4 + i + u * kThreads);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            f32x4 o;
            o.x = f(va[u].x, vb[u].x), o.y = f(va[u].y, vb[u].y), o.z = f(va[u].z, vb[u].z), o.w = f(va[u].w, vb[u].w);
            st_nt(r4 + i + u * kThreads, o);
        }
    }
    for (; i < n4; i += kThreads) {
        f32x4 va = a4[i], vb = b4[i], o;
        o.x = f(va.x, vb.x), o.y = f(va.y, vb.y), o.z = f(va.z, vb.z), o.w = f(va.w, vb.w);
        r4[i] = o;
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        long long t = (n4 << 2) + threadIdx.x;
        r[t] = f(a[t], b[t]);
    }
}

__global__ __launch_bounds__(kThreads) void vmul_kernel(const float* a, const float* b, float* r, long long n) {
    stream_binary(a, b, r, n, [](float x, float y) { return x * y; });
}
__global__ __launch_bounds__(kThreads) void vadd_kernel(const float* a, const float* b, float* r, long long n) {
    stream_binary(a, b, r, n, [](float x, float y) { return x + y; });
}
__global__ __launch_bounds__(kThreads) void axpy_kernel(float alpha, const float* x, float* y, long long n) {
    stream_binary(x, y, y, n, [alpha](float xv, float yv) { return fmaf(alpha, xv, yv); });
}

__global__ __launch_bounds__(kThreads) void fill_kernel(float* x, float v, long long n) {
    const long long stride = (long long)gridDim.x * kThreads;
    f32x4* x4 = reinterpret_cast<f32x4*>(x);
    const long long n4 = n >> 2;
    for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n4; i += stride) st_nt(x4 + i, f32x4{v, v, v, v});
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) x[(n4 << 2) + threadIdx.x] = v;
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kThreads) void rand_uniform_kernel(float* x, long long n, unsigned long long seed, float lo,
                                                               float scale) {
    const long long stride = (long long)gridDim.x * kThreads;
    for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
        unsigned long long h = mix64(seed * 0x9E3779B97F4A7C15ULL + (unsigned long long)i);
        float u = (float)(h >> 40) * (1.0f / 16777216.0f);  // 24 random bits -> [0,1)
        x[i] = lo + scale * u;
    }
}

// dst[i] = src[idx[i]] with 32-bit indices (the SpMV ghost exchange's send-buffer pack: per peer an ascending list of
// this rank's rows). Each thread packs 4 consecutive entries: one 16-B index load, 4 gathers through a buffer
// descriptor over src (an index outside [0, n_src) reads 0 instead of faulting), one 16-B store; the tail (n % 4)
// by the first block. torch.index_select with int64 indices moved 8 B of index per entry: 21 us -> (this) for the 5.2M
// entries of one N = 8 rank's step (scripts/spmv_host_lab.py).
__global__ __launch_bounds__(kThreads) void gather_kernel(const float* __restrict__ src, long long n_src,
                                                          const int* __restrict__ idx, float* __restrict__ dst,
                                                          long long n) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0,
                                                      (int)(n_src < (1LL << 29) ? n_src * 4 : 0x7ffffffc), 0x00020000);
    const long long n4 = n >> 2, stride = (long long)gridDim.x * kThreads;
    const pcmx::i32x4* idx4 = reinterpret_cast<const pcmx::i32x4*>(idx);
    f32x4* dst4 = reinterpret_cast<f32x4*>(dst);
    for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n4; i += stride) {
        const pcmx::i32x4 k = idx4[i];
        f32x4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            v[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (unsigned)k[q] * 4u, 0, 0));
        dst4[i] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const long long i = (n4 << 2) + threadIdx.x;
        dst[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (unsigned)idx[i] * 4u, 0, 0));
    }
}

inline int stream_grid(long long n, int per_thread) {
    long long blocks = ((n >> 2) + (long long)kThreads * per_thread - 1) / ((long long)kThreads * per_thread);
    if (blocks < 1) blocks = 1;
    if (blocks > pcmx::grid_cap_streaming()) blocks = pcmx::grid_cap_streaming();
    return (int)blocks;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }
}  // namespace

extern "C" int pcmx_vmul_f32(const float* a, const float* b, float* r, long long n, hipStream_t s) {
    if (n <= 0) return 0;
    if (!aligned16(a) || !aligned16(b) || !aligned16(r)) return -1;
    vmul_kernel<<<stream_grid(n, kUnroll), kThreads, 0, s>>>(a, b, r, n);
    return (int)hipGetLastError();
}

extern "C" int pcmx_vadd_f32(const float* a, const float* b, float* r, long long n, hipStream_t s) {
    if (n <= 0) return 0;
    if (!aligned16(a) || !aligned16(b) || !aligned16(r)) return -1;
    vadd_kernel<<<stream_grid(n, kUnroll), kThreads, 0, s>>>(a, b, r, n);
    return (int)hipGetLastError();
}

extern "C" int pcmx_axpy_f32(float alpha, const float* x, float* y, long long n, hipStream_t s) {
    if (n <= 0) return 0;
    if (!aligned16(x) || !aligned16(y)) return -1;
    axpy_kernel<<<stream_grid(n, kUnroll), kThreads, 0, s>>>(alpha, x, y, n);
    return (int)hipGetLastError();
}

extern "C" int pcmx_gather_f32(const float* src, long long n_src, const int* idx, float* dst, long long n,
                               hipStream_t s) {
    if (n <= 0) return 0;
    if (!aligned16(idx) || !aligned16(dst) || n_src <= 0 || n_src >= (1LL << 29)) return -1;
    gather_kernel<<<stream_grid(n, 1), kThreads, 0, s>>>(src, n_src, idx, dst, n);
    return (int)hipGetLastError();
}

extern "C" int pcmx_fill_f32(float* x, float v, long long n, hipStream_t s) {
    if (n <= 0) return 0;
    if (!aligned16(x)) return -1;
    fill_kernel<<<stream_grid(n, 1), kThreads, 0, s>>>(x, v, n);
    return (int)hipGetLastError();
}

extern "C" int pcmx_rand_uniform_f32(float* x, long long n, unsigned long long seed, float lo, float hi, hipStream_t s) {
    if (n <= 0) return 0;
    long long blocks = (n + kThreads - 1) / kThreads;
    if (blocks > pcmx::grid_cap_streaming()) blocks = pcmx::grid_cap_streaming();
    rand_uniform_kernel<<<(int)blocks, kThreads, 0, s>>>(x, n, seed, lo, hi - lo);
    return (int)hipGetLastError();
}
