// Global reductions (sum/min/max over f32 or i32, dot product) — the north-star "global reduction 1e9 f32"
// kernel and the device-side MIN flag of the distributed region growing (ref 2-mpi-region-growing/
// region.c:435-440, MPI_Allreduce MIN) before it goes to RCCL.
//
// Pass 1: grid capped at 256 CUs x 64 blocks, each thread keeps UNROLL independent float4 loads in flight
// (non-temporal: the data is streamed once), reduces in registers, then wave64 butterfly + LDS across the
// 4 waves. Pass 2: one block folds the <= 16384 partials in f64 (sum) in a fixed order, so the result is
// bitwise reproducible run to run (no float atomics, cdna_hip_programming.md G12). Grid cap (round 4,
// scripts/stream_bw_lab.hip, profiles/r4_bench/stream_bw_lab.txt): a 1e9-f32 read stream runs 6.70 TB/s with 2048
// blocks of 4 float4 per lane and 7.14 TB/s with 16384 (more blocks retire and refill the CUs' queues between
// each other's HBM round trips).
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
using pcmx::kWave;
constexpr int kThreads = 256;
constexpr int kUnroll = 4;  // float4 loads in flight per lane: 4 x 16 B x 256 threads = 16 KiB per block
constexpr int kMaxBlocks = 16384;

template <class T>
struct Vec4;
template <>
struct Vec4<float> {
    using type = pcmx::f32x4;
};
template <>
struct Vec4<int32_t> {
    using type = pcmx::i32x4;
};

template <class T, int OP>
__device__ __forceinline__ T identity() {
    if constexpr (OP == 0) return T(0);
    if constexpr (std::is_same<T, float>::value) return OP == 1 ? INFINITY : -INFINITY;
    return OP == 1 ? (T)0x7fffffff : (T)(-0x7fffffff - 1);
}

template <class T, int OP>
__device__ __forceinline__ T comb(T a, T b) {
    if constexpr (OP == 0) return a + b;
    if constexpr (OP == 1) return b < a ? b : a;
    return b > a ? b : a;
}

template <class T, int OP>
__device__ __forceinline__ T block_reduce(T v, T* lds) {
    v = pcmx::wave_reduce<T, OP>(v);
    const int w = threadIdx.x / kWave;
    if (pcmx::lane_id() == 0) lds[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        T r = lds[0];
        for (int i = 1; i < kThreads / kWave; ++i) r = comb<T, OP>(r, lds[i]);
        lds[0] = r;
    }
    __syncthreads();
    return lds[0];
}

// PROD=true: x*y element-wise product reduced with OP (dot product).
template <class T, int OP, bool PROD>
__global__ __launch_bounds__(kThreads) void reduce_pass1(const T* __restrict__ x, const T* __restrict__ y, long long n,
                                                        T* __restrict__ partials) {
    using V = typename Vec4<T>::type;
    __shared__ T lds[kThreads / kWave];
    const long long n4 = n >> 2;
    const V* x4 = reinterpret_cast<const V*>(x);
    const V* y4 = reinterpret_cast<const V*>(y);
    T acc[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) acc[u] = identity<T, OP>();
    const long long step = (long long)gridDim.x * kThreads * kUnroll;
    long long i = (long long)blockIdx.x * kThreads * kUnroll + threadIdx.x;
    for (; i + (kUnroll - 1) * kThreads < n4; i += step) {
        V v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) v[u] = __builtin_nontemporal_load(x4 + i + u * kThreads);
        if constexpr (PROD) {
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                V w = __builtin_nontemporal_load(y4 + i + u * kThreads);
                v[u].x *= w.x, v[u].y *= w.y, v[u].z *= w.z, v[u].w *= w.w;
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
            acc[u] = comb<T, OP>(acc[u], comb<T, OP>(comb<T, OP>(v[u].x, v[u].y), comb<T, OP>(v[u].z, v[u].w)));
    }
    for (; i < n4; i += kThreads) {
        V v = x4[i];
        if constexpr (PROD) {
            V w = y4[i];
            v.x *= w.x, v.y *= w.y, v.z *= w.z, v.w *= w.w;
        }
        acc[0] = comb<T, OP>(acc[0], comb<T, OP>(comb<T, OP>(v.x, v.y), comb<T, OP>(v.z, v.w)));
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        long long t = (n4 << 2) + threadIdx.x;
        T v = x[t];
        if constexpr (PROD) v *= y[t];
        acc[1] = comb<T, OP>(acc[1], v);
    }
#pragma unroll
    for (int u = 1; u < kUnroll; ++u) acc[0] = comb<T, OP>(acc[0], acc[u]);
    T r = block_reduce<T, OP>(acc[0], lds);
    if (threadIdx.x == 0) partials[blockIdx.x] = r;
}

// Fold the partials; sums are carried in a wider type (f64 for f32, i64 for i32) in a fixed order. All of up to
// 16384 partials are in flight at once (16 x 16-B loads per thread, one round trip; the former 8 scalar loads per
// thread took 8 dependent round trips, ~5 us), each thread folds its float4s in index order into 4 accumulators
// (one per component), so the result stays bitwise reproducible.
template <class T, int OP>
__global__ __launch_bounds__(kThreads) void reduce_pass2(const T* __restrict__ partials, int np, T* __restrict__ out) {
    using W = typename std::conditional<std::is_same<T, float>::value, double, long long>::type;
    using V = typename Vec4<T>::type;
    __shared__ W lds[kThreads / kWave];
    constexpr int kV = 16;  // float4s per thread per pass: 256 x 16 x 4 = 16384 partials (kMaxBlocks) in one pass
    const T id = identity<T, OP>();
    const W wid = OP == 0 ? W(0) : W(id);
    W acc[4] = {wid, wid, wid, wid};
    const int n4 = np >> 2;
    const V* p4 = reinterpret_cast<const V*>(partials);
    for (int base = 0; base < n4; base += kThreads * kV) {
        V v[kV];
#pragma unroll
        for (int u = 0; u < kV; ++u) {
            const int i = base + u * kThreads + (int)threadIdx.x;
            v[u] = i < n4 ? p4[i] : V{id, id, id, id};
        }
#pragma unroll
        for (int u = 0; u < kV; ++u) {
            acc[0] = comb<W, OP>(acc[0], (W)v[u][0]);
            acc[1] = comb<W, OP>(acc[1], (W)v[u][1]);
            acc[2] = comb<W, OP>(acc[2], (W)v[u][2]);
            acc[3] = comb<W, OP>(acc[3], (W)v[u][3]);
        }
    }
    if ((int)threadIdx.x < (np & 3)) acc[0] = comb<W, OP>(acc[0], (W)partials[(n4 << 2) + (int)threadIdx.x]);
    const W r = block_reduce<W, OP>(comb<W, OP>(comb<W, OP>(acc[0], acc[1]), comb<W, OP>(acc[2], acc[3])), lds);
    if (threadIdx.x == 0) out[0] = (T)r;
}

inline int pass1_blocks(long long n) {
    long long b = ((n >> 2) + (long long)kThreads * kUnroll - 1) / ((long long)kThreads * kUnroll);
    if (b < 1) b = 1;
    if (b > kMaxBlocks) b = kMaxBlocks;
    return (int)b;
}
inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

template <class T, bool PROD>
int launch_reduce(const T* x, const T* y, long long n, int op, T* out, void* ws, hipStream_t s) {
    if (n < 0 || !aligned16(x) || (PROD && !aligned16(y)) || ws == nullptr || !aligned16(ws)) return -1;
    const int nb = pass1_blocks(n);
    T* partials = reinterpret_cast<T*>(ws);
    switch (op) {
        case PCMX_OP_SUM:
            reduce_pass1<T, 0, PROD><<<nb, kThreads, 0, s>>>(x, y, n, partials);
            reduce_pass2<T, 0><<<1, kThreads, 0, s>>>(partials, nb, out);
            break;
        case PCMX_OP_MIN:
            reduce_pass1<T, 1, PROD><<<nb, kThreads, 0, s>>>(x, y, n, partials);
            reduce_pass2<T, 1><<<1, kThreads, 0, s>>>(partials, nb, out);
            break;
        case PCMX_OP_MAX:
            reduce_pass1<T, 2, PROD><<<nb, kThreads, 0, s>>>(x, y, n, partials);
            reduce_pass2<T, 2><<<1, kThreads, 0, s>>>(partials, nb, out);
            break;
        default:
            return -1;
    }
    return (int)hipGetLastError();
}
}  // namespace

extern "C" long long pcmx_reduce_workspace_bytes(long long n) { return (long long)pass1_blocks(n) * 8; }

extern "C" int pcmx_reduce_f32(const float* x, long long n, int op, float* out, void* ws, hipStream_t s) {
    return launch_reduce<float, false>(x, x, n, op, out, ws, s);
}
extern "C" int pcmx_reduce_i32(const int32_t* x, long long n, int op, int32_t* out, void* ws, hipStream_t s) {
    return launch_reduce<int32_t, false>(x, x, n, op, out, ws, s);
}
extern "C" int pcmx_dot_f32(const float* a, const float* b, long long n, float* out, void* ws, hipStream_t s) {
    return launch_reduce<float, true>(a, b, n, PCMX_OP_SUM, out, ws, s);
}
