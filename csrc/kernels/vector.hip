// Element-wise streaming kernels (HBM-bound): vmul (ref 6-opencl-region-growing/multiply_opencl.cl:1-4),
// vadd/axpy (north-star vector-add), copy, fill and on-device uniform random generation.
//
// MI355X design (round 6, scripts/stream_bw_lab.hip, profiles/r6_stream/): TICKET-ORDERED TILES. A persistent grid of
// one 512-thread block per CU takes 128-KiB tiles (per input) from an atomic ticket, double-buffered: the next tile's
// loads are issued before the current tile's stores (the streaming structure of scan_parked_kernel, scan.hip). Tiles
// then enter HBM in time order, so the whole chip streams one compact window of the arrays. Interleaved on one box
// (1e9 f32, nt loads and stores): copy 5.36-5.44 TB/s grid-stride -> 6.31-6.35 ticket; vadd 5.35-5.48 -> 6.44-6.51;
// axpy in place 5.27-5.37 -> 6.44-6.50. The same tiles handed out statically (tile = block + k * grid) stream at
// 5.06-5.13, so the ORDER is what pays, not the tile shape. The grid-stride form is box-dependent (5.4-6.6 TB/s on
// three boxes) where the ticket form held 6.31-6.38 on all three. (Round 4's "the write side tops out near 5.5 TB/s"
// was the grid-stride order on that box, not HBM.)
// The counter pair lives per (device, stream) and RESETS ITSELF: the last block to finish zeroes it, and stream order
// makes the next launch on that stream see zeros (no memset launch per call). During a hipGraph capture (no counter
// can be allocated, and a replay on another stream would share it) the launch takes the grid-stride form instead.
#include <map>
#include <mutex>
#include <utility>

#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
using pcmx::kWave;
constexpr int kThreads = 256;  // grid-stride fallback and the small kernels
constexpr int kUnroll = 4;
constexpr int kTileWaves = 8;  // ticket kernels: 512 threads, one block per CU

using pcmx::f32x4;
using pcmx::ld_nt;
using pcmx::st_nt;

struct Ticket {
    unsigned next;  // next tile to hand out
    unsigned done;  // blocks finished
};

// R f32x4 rows per lane and input: tile = 8 waves x 64 lanes x R float4s (R = 16: 128 KiB; two inputs take R = 8).
template <int R, int NIN>
struct Regs {
    f32x4 a[NIN >= 1 ? R : 1], b[NIN == 2 ? R : 1];
};

template <int R>
__device__ __forceinline__ long long tile_base(long long t) {
    return t * (kTileWaves * kWave * R) + (long long)(threadIdx.x / kWave) * (kWave * R) + (threadIdx.x & (kWave - 1));
}

template <int R, int NIN>
__device__ __forceinline__ void tile_load(const f32x4* a, const f32x4* b, long long n4, long long t, Regs<R, NIN>& v) {
    const long long base = tile_base<R>(t);
    const bool full = (t + 1) * (kTileWaves * kWave * R) <= n4;  // block-uniform
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long i = base + r * kWave;
        if constexpr (NIN >= 1) v.a[r] = (full || i < n4) ? ld_nt(a + i) : f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (NIN == 2) v.b[r] = (full || i < n4) ? ld_nt(b + i) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
}

template <int R, int NIN, class F>
__device__ __forceinline__ void tile_store(f32x4* out, long long n4, long long t, const Regs<R, NIN>& v, F f) {
    const long long base = tile_base<R>(t);
    const bool full = (t + 1) * (kTileWaves * kWave * R) <= n4;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long i = base + r * kWave;
        if (!(full || i < n4)) continue;
        f32x4 o;
        if constexpr (NIN == 2) {
            o.x = f(v.a[r].x, v.b[r].x), o.y = f(v.a[r].y, v.b[r].y), o.z = f(v.a[r].z, v.b[r].z), o.w = f(v.a[r].w, v.b[r].w);
        } else if constexpr (NIN == 1) {
            o.x = f(v.a[r].x, 0.f), o.y = f(v.a[r].y, 0.f), o.z = f(v.a[r].z, 0.f), o.w = f(v.a[r].w, 0.f);
        } else {
            const float c = f(0.f, 0.f);
            o = f32x4{c, c, c, c};
        }
        st_nt(out + i, o);
    }
}

// r[i] = f(a[i], b[i]) (NIN = 2), f(a[i], 0) (NIN = 1) or f(0, 0) (NIN = 0) over n floats; a / b / r 16-B aligned, r may
// alias an input element for element (axpy). Every block reaches the self-reset at the end (block-uniform exits).
template <int R, int NIN, class F>
__device__ __forceinline__ void stream_tiles(const float* a, const float* b, float* r, long long n, Ticket* tk, F f) {
    __shared__ unsigned s_t[2];
    const f32x4* a4 = reinterpret_cast<const f32x4*>(a);
    const f32x4* b4 = reinterpret_cast<const f32x4*>(b);
    f32x4* r4 = reinterpret_cast<f32x4*>(r);
    const long long n4 = n >> 2, tile4 = kTileWaves * kWave * R, ntiles = (n4 + tile4 - 1) / tile4;
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {  // the scalar tail (n % 4 floats)
        const long long t = (n4 << 2) + threadIdx.x;
        r[t] = f(NIN >= 1 ? a[t] : 0.f, NIN == 2 ? b[t] : 0.f);
    }
    auto take = [&](int slot) -> long long {
        if (threadIdx.x == 0) s_t[slot] = atomicAdd(&tk->next, 1u);
        __syncthreads();
        return (long long)s_t[slot];
    };
    Regs<R, NIN> va, vb;
    long long ta = take(0);
    if (ta < ntiles) {
        tile_load<R, NIN>(a4, b4, n4, ta, va);
        // unrolled by two so both register buffers are statically named; the next tile's loads go out before the
        // current tile's stores (vmcnt counts in issue order: the stores then wait only for their own tile)
        while (true) {
            const long long tb = take(1);
            if (tb < ntiles) tile_load<R, NIN>(a4, b4, n4, tb, vb);
            tile_store<R, NIN>(r4, n4, ta, va, f);
            if (tb >= ntiles) break;
            ta = take(0);
            if (ta < ntiles) tile_load<R, NIN>(a4, b4, n4, ta, va);
            tile_store<R, NIN>(r4, n4, tb, vb, f);
            if (ta >= ntiles) break;
        }
    }
    if (threadIdx.x == 0) {  // the last block to finish resets the pair for the next launch on this stream
        if (atomicAdd(&tk->done, 1u) == gridDim.x - 1) {
            atomicExch(&tk->next, 0u);
            atomicExch(&tk->done, 0u);
        }
    }
}

__global__ __launch_bounds__(kTileWaves * kWave) void vmul_tiles(const float* a, const float* b, float* r, long long n, Ticket* tk) {
    stream_tiles<8, 2>(a, b, r, n, tk, [](float x, float y) { return x * y; });
}
__global__ __launch_bounds__(kTileWaves * kWave) void vadd_tiles(const float* a, const float* b, float* r, long long n, Ticket* tk) {
    stream_tiles<8, 2>(a, b, r, n, tk, [](float x, float y) { return x + y; });
}
__global__ __launch_bounds__(kTileWaves * kWave) void axpy_tiles(float alpha, const float* x, float* y, long long n, Ticket* tk) {
    stream_tiles<8, 2>(x, y, y, n, tk, [alpha](float xv, float yv) { return fmaf(alpha, xv, yv); });
}
__global__ __launch_bounds__(kTileWaves * kWave) void copy_tiles(const float* a, float* r, long long n, Ticket* tk) {
    stream_tiles<16, 1>(a, nullptr, r, n, tk, [](float x, float) { return x; });
}
__global__ __launch_bounds__(kTileWaves * kWave) void fill_tiles(float* r, float v, long long n, Ticket* tk) {
    stream_tiles<16, 0>(nullptr, nullptr, r, n, tk, [v](float, float) { return v; });
}

// ---- grid-stride forms (hipGraph capture, and the reference point of the A/B)
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
__global__ __launch_bounds__(kThreads) void copy_kernel(const float* a, float* r, long long n) {
    stream_binary(a, a, r, n, [](float x, float) { return x; });
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

int device_cus() {  // cached per device (no attribute query on the launch path)
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus[dev] = 256;
    return cus[dev] > 0 ? cus[dev] : 256;
}

// The self-resetting counter pair of (device, stream), allocated and zeroed on first use (kept for the process);
// nullptr while `s` is capturing (the caller then launches the grid-stride form).
Ticket* stream_ticket(hipStream_t s) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, Ticket*> reg;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (cap != hipStreamCaptureStatusNone) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    auto it = reg.find({dev, s});
    if (it != reg.end()) return it->second;
    Ticket* t = nullptr;
    if (hipMalloc(&t, sizeof(Ticket)) != hipSuccess || hipMemset(t, 0, sizeof(Ticket)) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    reg[{dev, s}] = t;
    return t;
}

template <int R>
int tile_grid(long long n) {
    const long long tile = (long long)kTileWaves * kWave * R * 4, tiles = (n + tile - 1) / tile;
    const int cus = device_cus();
    return (int)(tiles < cus ? (tiles < 1 ? 1 : tiles) : cus);  // one resident 512-thread block per CU
}
}  // namespace

extern "C" int pcmx_vmul_f32(const float* a, const float* b, float* r, long long n, hipStream_t s) {
    if (n <= 0) return 0;
    if (!aligned16(a) || !aligned16(b) || !aligned16(r)) return -1;
    if (Ticket* tk = stream_ticket(s)) vmul_tiles<<<tile_grid<8>(n), kTileWaves * kWave, 0, s>>>(a, b, r, n, tk);
    else vmul_kernel<<<stream_grid(n, kUnroll), kThreads, 0, s>>>(a, b, r, n);
    return (int)hipGetLastError();
}

extern "C" int pcmx_vadd_f32(const float* a, const float* b, float* r, long long n, hipStream_t s) {
    if (n <= 0) return 0;
    if (!aligned16(a) || !aligned16(b) || !aligned16(r)) return -1;
    if (Ticket* tk = stream_ticket(s)) vadd_tiles<<<tile_grid<8>(n), kTileWaves * kWave, 0, s>>>(a, b, r, n, tk);
    else vadd_kernel<<<stream_grid(n, kUnroll), kThreads, 0, s>>>(a, b, r, n);
    return (int)hipGetLastError();
}

extern "C" int pcmx_axpy_f32(float alpha, const float* x, float* y, long long n, hipStream_t s) {
    if (n <= 0) return 0;
    if (!aligned16(x) || !aligned16(y)) return -1;
    if (Ticket* tk = stream_ticket(s)) axpy_tiles<<<tile_grid<8>(n), kTileWaves * kWave, 0, s>>>(alpha, x, y, n, tk);
    else axpy_kernel<<<stream_grid(n, kUnroll), kThreads, 0, s>>>(alpha, x, y, n);
    return (int)hipGetLastError();
}

extern "C" int pcmx_copy_f32(const float* a, float* r, long long n, hipStream_t s) {
    if (n <= 0) return 0;
    if (!aligned16(a) || !aligned16(r)) return -1;
    if (Ticket* tk = stream_ticket(s)) copy_tiles<<<tile_grid<16>(n), kTileWaves * kWave, 0, s>>>(a, r, n, tk);
    else copy_kernel<<<stream_grid(n, kUnroll), kThreads, 0, s>>>(a, r, n);
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
    if (Ticket* tk = stream_ticket(s)) fill_tiles<<<tile_grid<16>(n), kTileWaves * kWave, 0, s>>>(x, v, n, tk);
    else fill_kernel<<<stream_grid(n, 1), kThreads, 0, s>>>(x, v, n);
    return (int)hipGetLastError();
}

extern "C" int pcmx_rand_uniform_f32(float* x, long long n, unsigned long long seed, float lo, float hi, hipStream_t s) {
    if (n <= 0) return 0;
    long long blocks = (n + kThreads - 1) / kThreads;
    if (blocks > pcmx::grid_cap_streaming()) blocks = pcmx::grid_cap_streaming();
    rand_uniform_kernel<<<(int)blocks, kThreads, 0, s>>>(x, n, seed, lo, hi - lo);
    return (int)hipGetLastError();
}
